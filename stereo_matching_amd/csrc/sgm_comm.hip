// sgm_comm.hip -- the multi-GPU exchange of SURVEY.md 8e behind the C-ABI:
// stereo pairs shard one per GPU, and the only collective is the gather of
// the disparity maps to rank 0 (RCCL's ncclGather over xGMI).
//
// The reference has no multi-GPU path: node.cpp:49,93 makes one
// SGM::process call per pair on one object.  A C++ caller that owns several
// devices creates one sgm_handle per device and one communicator over them
// (sgm_comm_create: single process, ncclCommInitAll), runs a pair per device
// (one host thread per device, include/sgm_amd/BatchSGM.h), and gathers the
// maps with sgm_batch_gather[_all].  A job with one process per GPU (the
// torch.distributed.run layout bench.py uses) builds the same communicator
// from a unique id (sgm_comm_unique_id / sgm_comm_create_rank).
//
// RCCL is bound at run time (dlopen on the first sgm_comm_* call), not
// linked: a process that never gathers does not load it, and a process that
// already holds an RCCL -- the one PyTorch loads for its process groups --
// reuses that copy instead of mapping a second one beside it.
#include "../../include/sgm_hip.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <new>
#include <vector>

struct sgm_comm {
    int nranks;                     // ranks in the communicator
    int rank0;                      // global rank of local slot 0
    std::vector<int> dev;           // device of each local slot
    std::vector<ncclComm_t> comm;   // RCCL communicator of each local slot
    std::vector<float *> stage;     // per slot: packed copy of a pitched map (lazy)
    std::vector<size_t> stage_n;    //   its size in floats
    char err[256];
};

namespace {

struct Rccl {
    void *so = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGather) gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

std::mutex g_mu;
Rccl g_rccl;
// errors before a communicator exists (sgm_comm_last_error(NULL)), per
// calling thread: BatchSGM-style callers create and gather from several
thread_local char g_err[256];

void set_gerr(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int set_cerr(sgm_comm *c, int code, const char *fmt, ...) {
    char *dst = c ? c->err : g_err;
    const size_t n = c ? sizeof(c->err) : sizeof(g_err);
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(dst, n, fmt, ap);
    va_end(ap);
    return code;
}

// The RCCL this process uses: SGM_RCCL_LIB if set; else one already loaded
// (PyTorch's librccl.so carries no soname, /opt/rocm's is librccl.so.1);
// else /opt/rocm's, loaded with its own symbols first (RTLD_DEEPBIND), so it
// never binds into another copy's internals.
const Rccl *rccl() {
    std::lock_guard<std::mutex> lock(g_mu);
    if (g_rccl.so) return &g_rccl;
    void *so = nullptr;
    const char *env = getenv("SGM_RCCL_LIB");
    if (env && *env) {
        so = dlopen(env, RTLD_NOW | RTLD_LOCAL);
        if (!so) {
            set_gerr("dlopen(SGM_RCCL_LIB=%s) failed: %s", env, dlerror());
            return nullptr;
        }
    } else {
        const char *loaded[] = {"librccl.so", "librccl.so.1"};
        for (const char *name : loaded)
            if (!so) so = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
        const char *fresh[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"};
        for (const char *name : fresh)
            if (!so) so = dlopen(name, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
        if (!so) {
            set_gerr("RCCL (librccl.so.1) could not be loaded: %s", dlerror());
            return nullptr;
        }
    }
    Rccl r;
    r.so = so;
    bool ok = true;
    auto sym = [&](auto &fn, const char *name) {
        fn = reinterpret_cast<typename std::remove_reference<decltype(fn)>::type>(dlsym(so, name));
        if (!fn) {
            set_gerr("RCCL lacks %s", name);
            ok = false;
        }
    };
    sym(r.get_unique_id, "ncclGetUniqueId");
    sym(r.init_rank, "ncclCommInitRank");
    sym(r.init_all, "ncclCommInitAll");
    sym(r.destroy, "ncclCommDestroy");
    sym(r.gather, "ncclGather");
    sym(r.group_start, "ncclGroupStart");
    sym(r.group_end, "ncclGroupEnd");
    sym(r.error_string, "ncclGetErrorString");
    if (!ok) return nullptr;  // (the handle stays open: dlclose of an RCCL is unsafe)
    g_rccl = r;
    return &g_rccl;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

int check_devices(const int *devices, int n, char *why, size_t len) {
    if (!devices || n <= 0) {
        snprintf(why, len, "devices must list n > 0 HIP ordinals");
        return SGM_ERR_INVALID_ARG;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        snprintf(why, len, "no HIP device");
        return SGM_ERR_NO_DEVICE;
    }
    for (int i = 0; i < n; ++i) {
        if (devices[i] < 0 || devices[i] >= ndev) {
            snprintf(why, len, "devices[%d] = %d is not a HIP ordinal (0..%d)", i, devices[i], ndev - 1);
            return SGM_ERR_INVALID_ARG;
        }
        for (int k = 0; k < i; ++k)
            if (devices[k] == devices[i]) {
                // (RCCL holds one rank per device)
                snprintf(why, len, "device %d is listed twice", devices[i]);
                return SGM_ERR_INVALID_ARG;
            }
    }
    return SGM_OK;
}

void free_comm(sgm_comm *c, const Rccl *r) {
    for (size_t s = 0; s < c->comm.size(); ++s) {
        DeviceGuard guard(c->dev[s]);
        if (c->comm[s] && r) (void)r->destroy(c->comm[s]);
        if (c->stage[s]) (void)hipFree(c->stage[s]);
    }
    delete c;
}

sgm_comm *new_comm(int nlocal) {
    sgm_comm *c = new (std::nothrow) sgm_comm();
    if (!c) return nullptr;
    c->dev.assign(nlocal, -1);
    c->comm.assign(nlocal, nullptr);
    c->stage.assign(nlocal, nullptr);
    c->stage_n.assign(nlocal, 0);
    c->err[0] = 0;
    return c;
}

// One rank's ncclGather, enqueued on `stream` (its device current).
int gather_one(sgm_comm *c, const Rccl *r, int slot, const float *d_map, int rows, int cols, int pitch,
               float *d_root_out, hipStream_t st) {
    const size_t n = (size_t)rows * cols;
    const float *send = d_map;
    if (pitch != cols) {  // RCCL sends one contiguous range: pack the rows
        if (c->stage_n[slot] < n) {
            if (c->stage[slot]) (void)hipFree(c->stage[slot]);
            c->stage[slot] = nullptr;
            c->stage_n[slot] = 0;
            hipError_t e = hipMalloc((void **)&c->stage[slot], n * sizeof(float));
            if (e != hipSuccess)
                return set_cerr(c, e == hipErrorOutOfMemory ? SGM_ERR_OUT_OF_MEMORY : SGM_ERR_HIP,
                                "sgm_batch_gather: staging buffer: %s", hipGetErrorString(e));
            c->stage_n[slot] = n;
        }
        hipError_t e = hipMemcpy2DAsync(c->stage[slot], (size_t)cols * sizeof(float), d_map,
                                        (size_t)pitch * sizeof(float), (size_t)cols * sizeof(float), rows,
                                        hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess)
            return set_cerr(c, SGM_ERR_HIP, "sgm_batch_gather: packing the map: %s", hipGetErrorString(e));
        send = c->stage[slot];
    }
    const int rank = c->rank0 + slot;
    ncclResult_t nr = r->gather(send, rank == 0 ? d_root_out : nullptr, n, ncclFloat32, 0, c->comm[slot], st);
    if (nr != ncclSuccess)
        return set_cerr(c, SGM_ERR_HIP, "ncclGather (rank %d): %s", rank, r->error_string(nr));
    return SGM_OK;
}

int check_gather_args(sgm_comm *c, const float *d_map, int rows, int cols, int pitch, bool root,
                      const float *d_root_out) {
    if (!d_map || rows <= 0 || cols <= 0 || pitch < cols)
        return set_cerr(c, SGM_ERR_INVALID_ARG, "sgm_batch_gather: bad map pointer, size or pitch");
    if ((size_t)rows * cols * (size_t)c->nranks > ((size_t)1 << 40))
        return set_cerr(c, SGM_ERR_INVALID_ARG, "sgm_batch_gather: maps too large");
    if (root && !d_root_out)
        return set_cerr(c, SGM_ERR_INVALID_ARG, "sgm_batch_gather: rank 0 needs d_root_out");
    return SGM_OK;
}

}  // namespace

extern "C" {

int sgm_comm_create(const int *devices, int n, sgm_comm **out) {
    if (!out) return set_cerr(nullptr, SGM_ERR_INVALID_ARG, "sgm_comm_create: out is NULL");
    *out = nullptr;
    char why[160];
    if (int rc = check_devices(devices, n, why, sizeof(why))) return set_cerr(nullptr, rc, "sgm_comm_create: %s", why);
    const Rccl *r = rccl();
    if (!r) return SGM_ERR_HIP;
    sgm_comm *c = new_comm(n);
    if (!c) return set_cerr(nullptr, SGM_ERR_OUT_OF_MEMORY, "sgm_comm_create: out of host memory");
    c->nranks = n;
    c->rank0 = 0;
    for (int i = 0; i < n; ++i) c->dev[i] = devices[i];
    int prev = -1;
    (void)hipGetDevice(&prev);
    ncclResult_t nr = r->init_all(c->comm.data(), n, devices);
    if (prev >= 0) (void)hipSetDevice(prev);
    if (nr != ncclSuccess) {
        set_cerr(nullptr, SGM_ERR_HIP, "ncclCommInitAll over %d devices: %s", n, r->error_string(nr));
        for (auto &cm : c->comm) cm = nullptr;
        free_comm(c, r);
        return SGM_ERR_HIP;
    }
    *out = c;
    return SGM_OK;
}

int sgm_comm_unique_id(char id[SGM_COMM_ID_BYTES]) {
    if (!id) return set_cerr(nullptr, SGM_ERR_INVALID_ARG, "sgm_comm_unique_id: id is NULL");
    const Rccl *r = rccl();
    if (!r) return SGM_ERR_HIP;
    static_assert(sizeof(ncclUniqueId) == SGM_COMM_ID_BYTES, "unique id size");
    ncclUniqueId u;
    ncclResult_t nr = r->get_unique_id(&u);
    if (nr != ncclSuccess) return set_cerr(nullptr, SGM_ERR_HIP, "ncclGetUniqueId: %s", r->error_string(nr));
    memcpy(id, &u, sizeof(u));
    return SGM_OK;
}

int sgm_comm_create_rank(const char id[SGM_COMM_ID_BYTES], int nranks, int rank, int device, sgm_comm **out) {
    if (!out) return set_cerr(nullptr, SGM_ERR_INVALID_ARG, "sgm_comm_create_rank: out is NULL");
    *out = nullptr;
    if (!id || nranks <= 0 || rank < 0 || rank >= nranks)
        return set_cerr(nullptr, SGM_ERR_INVALID_ARG, "sgm_comm_create_rank: bad id, nranks or rank");
    char why[160];
    if (int rc = check_devices(&device, 1, why, sizeof(why)))
        return set_cerr(nullptr, rc, "sgm_comm_create_rank: %s", why);
    const Rccl *r = rccl();
    if (!r) return SGM_ERR_HIP;
    sgm_comm *c = new_comm(1);
    if (!c) return set_cerr(nullptr, SGM_ERR_OUT_OF_MEMORY, "sgm_comm_create_rank: out of host memory");
    c->nranks = nranks;
    c->rank0 = rank;
    c->dev[0] = device;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclResult_t nr;
    {
        DeviceGuard guard(device);
        nr = r->init_rank(&c->comm[0], nranks, u, rank);
    }
    if (nr != ncclSuccess) {
        set_cerr(nullptr, SGM_ERR_HIP, "ncclCommInitRank (rank %d of %d): %s", rank, nranks, r->error_string(nr));
        c->comm[0] = nullptr;
        free_comm(c, r);
        return SGM_ERR_HIP;
    }
    *out = c;
    return SGM_OK;
}

int sgm_comm_destroy(sgm_comm *c) {
    if (!c) return SGM_ERR_INVALID_ARG;
    free_comm(c, rccl());
    return SGM_OK;
}

const char *sgm_comm_last_error(const sgm_comm *c) { return c ? c->err : g_err; }

int sgm_comm_info(const sgm_comm *c, int *nranks, int *first_rank, int *nlocal) {
    if (!c) return SGM_ERR_INVALID_ARG;
    if (nranks) *nranks = c->nranks;
    if (first_rank) *first_rank = c->rank0;
    if (nlocal) *nlocal = (int)c->comm.size();
    return SGM_OK;
}

int sgm_batch_gather(sgm_comm *c, int rank, const float *d_map, int rows, int cols, int pitch,
                     float *d_root_out, void *stream) {
    if (!c) return SGM_ERR_INVALID_ARG;
    const int slot = rank - c->rank0;
    if (slot < 0 || slot >= (int)c->comm.size())
        return set_cerr(c, SGM_ERR_INVALID_ARG, "sgm_batch_gather: rank %d is not held by this communicator "
                        "(ranks %d..%d)", rank, c->rank0, c->rank0 + (int)c->comm.size() - 1);
    if (int rc = check_gather_args(c, d_map, rows, cols, pitch, rank == 0, d_root_out)) return rc;
    const Rccl *r = rccl();
    if (!r) return set_cerr(c, SGM_ERR_HIP, "%s", g_err);
    DeviceGuard guard(c->dev[slot]);
    return gather_one(c, r, slot, d_map, rows, cols, pitch, d_root_out, (hipStream_t)stream);
}

int sgm_batch_gather_all(sgm_comm *c, const float *const *d_maps, int rows, int cols, int pitch,
                         float *d_root_out, void *const *streams) {
    if (!c) return SGM_ERR_INVALID_ARG;
    if (!d_maps) return set_cerr(c, SGM_ERR_INVALID_ARG, "sgm_batch_gather_all: d_maps is NULL");
    const int nlocal = (int)c->comm.size();
    for (int s = 0; s < nlocal; ++s)
        if (int rc = check_gather_args(c, d_maps[s], rows, cols, pitch, c->rank0 + s == 0, d_root_out)) return rc;
    const Rccl *r = rccl();
    if (!r) return set_cerr(c, SGM_ERR_HIP, "%s", g_err);
    // one thread drives every local rank: the ranks' calls form one group
    // (ncclGroupStart/End), or the first would wait for the others forever
    ncclResult_t nr = r->group_start();
    if (nr != ncclSuccess) return set_cerr(c, SGM_ERR_HIP, "ncclGroupStart: %s", r->error_string(nr));
    int rc = SGM_OK;
    for (int s = 0; s < nlocal && rc == SGM_OK; ++s) {
        DeviceGuard guard(c->dev[s]);
        rc = gather_one(c, r, s, d_maps[s], rows, cols, pitch, d_root_out,
                        streams ? (hipStream_t)streams[s] : (hipStream_t)0);
    }
    nr = r->group_end();
    if (rc) return rc;
    if (nr != ncclSuccess) return set_cerr(c, SGM_ERR_HIP, "ncclGroupEnd: %s", r->error_string(nr));
    return SGM_OK;
}

}  // extern "C"
