/*
 * sgm_amd/BatchSGM.h -- a batch of stereo pairs over several MI355X GPUs from
 * C++, one pair per device, maps gathered to the first device by RCCL over
 * xGMI (BASELINE.json config 4: 8 KITTI pairs on 8 GPUs).
 *
 * The reference has no multi-GPU path: the ROS node builds one SGM and calls
 * process(l, r) / get_disp() per pair (node.cpp:49,93,104).  BatchSGM holds
 * that object once per device -- an sgm_handle with the same parameters as
 * sgm_amd::SGM (both views, LR check, post_filter: get_disp()'s map) -- and
 * runs pair k of a batch on device k % n, one host thread per device, in
 * rounds of n pairs.  After each round's frames every thread calls sgm_check
 * (a frame whose slanted-pass hand-off gave up is never gathered), then one
 * sgm_batch_gather_all moves the round's maps into the first device's
 * buffer (ncclGather, root 0) and from there into pinned host memory, from
 * where they are copied to get_disp(k).  The only exchange is that gather:
 * no collective on the data path.
 *
 * Batches larger than n overlap: each device's map and the root buffer are
 * double-buffered, and round r's gather and device-to-host copy run on
 * per-device gather streams while round r+1's frames run on the handles'
 * streams.  A device without a pair in a (last, partial) round sends a
 * zeroed map, which is gathered but never copied out.
 *
 * Header-only, C++11, with the HIP runtime API on the host side (compile
 * with -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include and link -lsgm_hip
 * -lamdhip64 -pthread).  Errors go through sgm_amd::fail (abort, or
 * std::runtime_error with SGM_AMD_THROW), as the class surface's do.
 */
#ifndef SGM_AMD_BATCH_SGM_H
#define SGM_AMD_BATCH_SGM_H

#include <hip/hip_runtime_api.h>

#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../sgm_hip.h"
#include "SGM.h"

namespace sgm_amd {

class BatchSGM {
public:
    // SGM(h, w, s, d) (node.cpp:49) on every device of `devices` (HIP
    // ordinals, each once), in one communicator (sgm_comm_create).
    BatchSGM(const std::vector<int> &devices, int h, int w, int s, int d) : in_h_(h), in_w_(w) {
        if (devices.empty()) fail("BatchSGM", "no devices");
        sgm_params p;
        if (sgm_default_params(&p, h, w, s, d) != SGM_OK) fail("BatchSGM", "sgm_default_params");
        p.post_filter = 1;  // get_disp(): LR check + post_filter (SGM.cpp:803-821), as sgm_amd::SGM
        slots_.resize(devices.size());
        for (size_t k = 0; k < devices.size(); ++k) {
            Slot &sl = slots_[k];
            sl.device = devices[k];
            if (sgm_create(&p, sl.device, &sl.h) != SGM_OK) {
                release();
                fail("BatchSGM", "sgm_create failed (see stderr)");
            }
            sgm_get_size(sl.h, &rows_, &cols_, nullptr);
            sl.stream = sgm_get_stream(sl.h);
            ctor_hip(hipSetDevice(sl.device), "hipSetDevice");
            ctor_hip(hipMalloc(&sl.d_l, (size_t)h * w), "hipMalloc");
            ctor_hip(hipMalloc(&sl.d_r, (size_t)h * w), "hipMalloc");
            ctor_hip(hipStreamCreateWithFlags(&sl.gstream, hipStreamNonBlocking), "hipStreamCreate");
            for (int b = 0; b < 2; ++b) {
                ctor_hip(hipMalloc(&sl.d_map[b], map_bytes()), "hipMalloc");
                // defined contents from the start (an idle device's map is gathered too)
                ctor_hip(hipMemset(sl.d_map[b], 0, map_bytes()), "hipMemset");
                ctor_hip(hipEventCreateWithFlags(&sl.ev_gathered[b], hipEventDisableTiming), "hipEventCreate");
            }
        }
        if (sgm_comm_create(devices.data(), (int)devices.size(), &comm_) != SGM_OK) {
            const std::string why = sgm_comm_last_error(nullptr);
            release();
            fail("sgm_comm_create", why.c_str());
        }
        ctor_hip(hipSetDevice(devices[0]), "hipSetDevice");
        for (int b = 0; b < 2; ++b) {
            ctor_hip(hipMalloc(&d_root_[b], devices.size() * map_bytes()), "hipMalloc");
            ctor_hip(hipHostMalloc((void **)&h_stage_[b], devices.size() * map_bytes(), hipHostMallocDefault),
                     "hipHostMalloc");
            ctor_hip(hipEventCreateWithFlags(&ev_copied_[b], hipEventDisableTiming), "hipEventCreate");
        }
    }
    ~BatchSGM() { release(); }
    BatchSGM(const BatchSGM &) = delete;
    BatchSGM &operator=(const BatchSGM &) = delete;

    int devices() const { return (int)slots_.size(); }

    // process(left[k], right[k]) for every pair k (node.cpp:93); afterwards
    // get_disp(k) is pair k's map (CV_32FC1, rows x cols, invalid = d+1).
    void process(const std::vector<Mat> &left, const std::vector<Mat> &right) {
        check_batch(left, right, in_h_, in_w_);
        const size_t n = slots_.size();
        disp_.resize(left.size());
        size_t prev_first = 0, prev_count = 0;
        int prev_b = -1;
        for (size_t first = 0, round = 0; first < left.size(); first += n, ++round) {
            const size_t count = round_count(left.size(), first, n);
            const int b = (int)(round & 1);
            // one host thread per device: its pair's frame into map buffer b
            // (after the gather two rounds back has read it), then sgm_check;
            // a device without a pair zeroes buffer b instead
            std::vector<std::thread> th;
            for (size_t k = 0; k < n; ++k)
                th.emplace_back([this, k, b, first, count, &left, &right] {
                    if (k < count) run_slot(slots_[k], b, left[first + k], right[first + k]);
                    else zero_slot(slots_[k], b);
                });
            for (auto &t : th) t.join();
            for (size_t k = 0; k < n; ++k)
                if (!slots_[k].error.empty()) {
                    drain();
                    fail("BatchSGM::process", slots_[k].error.c_str());
                }
            // the round's maps to the first device and on to pinned host
            // memory, on the gather streams: they run under the next round's
            // frames (the root buffer b's previous copy-out is ahead of this
            // gather on the first device's gather stream)
            std::vector<const float *> maps(n);
            std::vector<void *> streams(n);
            for (size_t k = 0; k < n; ++k) {
                maps[k] = slots_[k].d_map[b];
                streams[k] = slots_[k].gstream;
            }
            if (sgm_batch_gather_all(comm_, maps.data(), rows_, cols_, cols_, d_root_[b], streams.data()) != SGM_OK) {
                drain();
                fail("sgm_batch_gather_all", sgm_comm_last_error(comm_));
            }
            for (size_t k = 0; k < n; ++k) {
                check_hip(hipSetDevice(slots_[k].device), "hipSetDevice");
                check_hip(hipEventRecord(slots_[k].ev_gathered[b], slots_[k].gstream), "hipEventRecord");
            }
            check_hip(hipSetDevice(slots_[0].device), "hipSetDevice");
            check_hip(hipMemcpyAsync(h_stage_[b], d_root_[b], count * map_bytes(), hipMemcpyDeviceToHost,
                                     slots_[0].gstream),
                      "hipMemcpyAsync");
            check_hip(hipEventRecord(ev_copied_[b], slots_[0].gstream), "hipEventRecord");
            if (prev_b >= 0) copy_out(prev_b, prev_first, prev_count);
            prev_b = b;
            prev_first = first;
            prev_count = count;
        }
        if (prev_b >= 0) copy_out(prev_b, prev_first, prev_count);
    }

    const Mat &get_disp(int k) const {
        if (k < 0 || k >= (int)disp_.size()) fail("BatchSGM::get_disp", "no such pair");
        return disp_[k];
    }

    // pairs in the round that starts at pair `first` of `total`, n devices
    static size_t round_count(size_t total, size_t first, size_t n) {
        return total - first < n ? total - first : n;
    }

    // process()'s argument checks (no device work): equal counts, CV_8UC1
    // inputs of the constructed size (SGM.cpp:34-38)
    static void check_batch(const std::vector<Mat> &left, const std::vector<Mat> &right, int h, int w) {
        if (left.size() != right.size()) fail("BatchSGM::process", "left and right counts differ");
        for (size_t k = 0; k < left.size(); ++k)
            if (left[k].type() != CV_8UC1 || right[k].type() != CV_8UC1 || left[k].rows != h ||
                left[k].cols != w || right[k].rows != h || right[k].cols != w)
                fail("BatchSGM::process", "inputs must be CV_8UC1 of the constructed size (SGM.cpp:34-38)");
    }

private:
    struct Slot {
        int device = -1;
        sgm_handle *h = nullptr;
        void *stream = nullptr;            // the handle's stream: uploads and frames
        hipStream_t gstream = nullptr;     // gathers (and, on the first device, copies out)
        unsigned char *d_l = nullptr, *d_r = nullptr;
        float *d_map[2] = {nullptr, nullptr};
        hipEvent_t ev_gathered[2] = {nullptr, nullptr};  // the last gather of d_map[b] is done
        std::string error;
    };
    std::vector<Slot> slots_;
    sgm_comm *comm_ = nullptr;
    float *d_root_[2] = {nullptr, nullptr};
    float *h_stage_[2] = {nullptr, nullptr};
    hipEvent_t ev_copied_[2] = {nullptr, nullptr};
    int in_h_, in_w_, rows_ = 0, cols_ = 0;
    std::vector<Mat> disp_;

    size_t map_bytes() const { return (size_t)rows_ * cols_ * sizeof(float); }

    static void check_hip(hipError_t e, const char *what) {
        if (e != hipSuccess) fail(what, hipGetErrorString(e));
    }
    // the constructor's: release what exists before failing
    void ctor_hip(hipError_t e, const char *what) {
        if (e != hipSuccess) {
            const std::string why = hipGetErrorString(e);
            release();
            fail(what, why.c_str());
        }
    }

    // one pair on one device (a worker thread): upload, frame, sgm_check
    static void run_slot(Slot &sl, int b, const Mat &l, const Mat &r) {
        sl.error.clear();
        hipStream_t st = (hipStream_t)sl.stream;
        const size_t w = (size_t)l.cols;
        if (hipSetDevice(sl.device) != hipSuccess || hipStreamWaitEvent(st, sl.ev_gathered[b], 0) != hipSuccess ||
            hipMemcpy2DAsync(sl.d_l, w, l.data, (size_t)l.step, w, l.rows, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpy2DAsync(sl.d_r, w, r.data, (size_t)r.step, w, r.rows, hipMemcpyHostToDevice, st) != hipSuccess) {
            sl.error = "uploading the pair failed";
            return;
        }
        int rows = 0, cols = 0;
        sgm_get_size(sl.h, &rows, &cols, nullptr);
        // NULL stream: the handle's own (sl.stream), where the upload went
        if (sgm_process_device(sl.h, sl.d_l, sl.d_r, l.cols, nullptr, nullptr, 0, sl.d_map[b], cols, nullptr,
                               nullptr) != SGM_OK ||
            sgm_check(sl.h) != SGM_OK)
            sl.error = sgm_last_error(sl.h);
    }

    // a device without a pair this round: a zeroed map (defined bytes in the gather)
    void zero_slot(Slot &sl, int b) {
        sl.error.clear();
        if (hipSetDevice(sl.device) != hipSuccess ||
            hipMemsetAsync(sl.d_map[b], 0, map_bytes(), sl.gstream) != hipSuccess)
            sl.error = "zeroing an idle device's map failed";
    }

    // a finished round's maps from pinned host memory into get_disp's Mats
    void copy_out(int b, size_t first, size_t count) {
        check_hip(hipSetDevice(slots_[0].device), "hipSetDevice");
        check_hip(hipEventSynchronize(ev_copied_[b]), "hipEventSynchronize");
        for (size_t k = 0; k < count; ++k) {
            Mat &m = disp_[first + k];
            m.create(rows_, cols_, CV_32FC1);
            const float *src = h_stage_[b] + k * (size_t)rows_ * cols_;
            for (int i = 0; i < rows_; ++i)
                std::memcpy(m.ptr<float>(i), src + (size_t)i * cols_, (size_t)cols_ * sizeof(float));
        }
    }

    // before failing mid-batch: no gather or copy may still use the buffers
    void drain() {
        for (auto &sl : slots_)
            if (sl.device >= 0 && hipSetDevice(sl.device) == hipSuccess) (void)hipDeviceSynchronize();
    }

    void release() {
        if (comm_) sgm_comm_destroy(comm_);
        comm_ = nullptr;
        if (!slots_.empty() && slots_[0].device >= 0) {
            (void)hipSetDevice(slots_[0].device);
            (void)hipDeviceSynchronize();
            for (int b = 0; b < 2; ++b) {
                if (d_root_[b]) (void)hipFree(d_root_[b]);
                if (h_stage_[b]) (void)hipHostFree(h_stage_[b]);
                if (ev_copied_[b]) (void)hipEventDestroy(ev_copied_[b]);
                d_root_[b] = nullptr;
                h_stage_[b] = nullptr;
                ev_copied_[b] = nullptr;
            }
        }
        for (auto &sl : slots_) {
            if (sl.device >= 0) {
                (void)hipSetDevice(sl.device);
                (void)hipDeviceSynchronize();
            }
            if (sl.d_l) (void)hipFree(sl.d_l);
            if (sl.d_r) (void)hipFree(sl.d_r);
            for (int b = 0; b < 2; ++b) {
                if (sl.d_map[b]) (void)hipFree(sl.d_map[b]);
                if (sl.ev_gathered[b]) (void)hipEventDestroy(sl.ev_gathered[b]);
            }
            if (sl.gstream) (void)hipStreamDestroy(sl.gstream);
            if (sl.h) sgm_destroy(sl.h);
            sl = Slot();
        }
    }
};

}  // namespace sgm_amd

#endif
