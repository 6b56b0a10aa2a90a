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
 * buffer (ncclGather, root 0), from where they are copied to get_disp(k).
 * The only exchange is that gather: no collective on the data path.
 *
 * Header-only, C++11, with the HIP runtime API on the host side (compile
 * with -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include and link -lsgm_hip
 * -lamdhip64 -pthread).  Errors go through sgm_amd::fail (abort, or
 * std::runtime_error with SGM_AMD_THROW), as the class surface's do.
 */
#ifndef SGM_AMD_BATCH_SGM_H
#define SGM_AMD_BATCH_SGM_H

#include <hip/hip_runtime_api.h>

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
            check_hip(hipSetDevice(sl.device), "hipSetDevice");
            check_hip(hipMalloc(&sl.d_l, (size_t)h * w), "hipMalloc");
            check_hip(hipMalloc(&sl.d_r, (size_t)h * w), "hipMalloc");
            check_hip(hipMalloc(&sl.d_map, (size_t)rows_ * cols_ * sizeof(float)), "hipMalloc");
        }
        if (sgm_comm_create(devices.data(), (int)devices.size(), &comm_) != SGM_OK) {
            const std::string why = sgm_comm_last_error(nullptr);
            release();
            fail("sgm_comm_create", why.c_str());
        }
        check_hip(hipSetDevice(devices[0]), "hipSetDevice");
        check_hip(hipMalloc(&d_root_, devices.size() * (size_t)rows_ * cols_ * sizeof(float)), "hipMalloc");
    }
    ~BatchSGM() { release(); }
    BatchSGM(const BatchSGM &) = delete;
    BatchSGM &operator=(const BatchSGM &) = delete;

    int devices() const { return (int)slots_.size(); }

    // process(left[k], right[k]) for every pair k (node.cpp:93); afterwards
    // get_disp(k) is pair k's map (CV_32FC1, rows x cols, invalid = d+1).
    void process(const std::vector<Mat> &left, const std::vector<Mat> &right) {
        if (left.size() != right.size()) fail("BatchSGM::process", "left and right counts differ");
        for (size_t k = 0; k < left.size(); ++k)
            if (left[k].type() != CV_8UC1 || right[k].type() != CV_8UC1 || left[k].rows != in_h_ ||
                left[k].cols != in_w_ || right[k].rows != in_h_ || right[k].cols != in_w_)
                fail("BatchSGM::process", "inputs must be CV_8UC1 of the constructed size (SGM.cpp:34-38)");
        const size_t n = slots_.size();
        disp_.resize(left.size());
        for (size_t first = 0; first < left.size(); first += n) {
            const size_t count = left.size() - first < n ? left.size() - first : n;
            // one host thread per device: its pair's frame, then sgm_check
            std::vector<std::thread> th;
            for (size_t k = 0; k < count; ++k)
                th.emplace_back([this, k, first, &left, &right] {
                    run_slot(slots_[k], left[first + k], right[first + k]);
                });
            for (auto &t : th) t.join();
            for (size_t k = 0; k < count; ++k)
                if (!slots_[k].error.empty()) fail("BatchSGM::process", slots_[k].error.c_str());
            // the round's maps to the first device (ranks without a pair this
            // round send their previous map; it is not read)
            std::vector<const float *> maps(n);
            std::vector<void *> streams(n);
            for (size_t k = 0; k < n; ++k) {
                maps[k] = slots_[k].d_map;
                streams[k] = slots_[k].stream;
            }
            if (sgm_batch_gather_all(comm_, maps.data(), rows_, cols_, cols_, d_root_, streams.data()) != SGM_OK)
                fail("sgm_batch_gather_all", sgm_comm_last_error(comm_));
            check_hip(hipSetDevice(slots_[0].device), "hipSetDevice");
            check_hip(hipStreamSynchronize((hipStream_t)slots_[0].stream), "hipStreamSynchronize");
            for (size_t k = 0; k < count; ++k) {
                Mat &m = disp_[first + k];
                m.create(rows_, cols_, CV_32FC1);
                check_hip(hipMemcpy2D(m.data, (size_t)m.step, d_root_ + k * (size_t)rows_ * cols_,
                                      (size_t)cols_ * sizeof(float), (size_t)cols_ * sizeof(float), rows_,
                                      hipMemcpyDeviceToHost),
                          "hipMemcpy2D");
            }
        }
    }

    const Mat &get_disp(int k) const {
        if (k < 0 || k >= (int)disp_.size()) fail("BatchSGM::get_disp", "no such pair");
        return disp_[k];
    }

private:
    struct Slot {
        int device = -1;
        sgm_handle *h = nullptr;
        void *stream = nullptr;
        unsigned char *d_l = nullptr, *d_r = nullptr;
        float *d_map = nullptr;
        std::string error;
    };
    std::vector<Slot> slots_;
    sgm_comm *comm_ = nullptr;
    float *d_root_ = nullptr;
    int in_h_, in_w_, rows_ = 0, cols_ = 0;
    std::vector<Mat> disp_;

    static void check_hip(hipError_t e, const char *what) {
        if (e != hipSuccess) fail(what, hipGetErrorString(e));
    }

    // one pair on one device (a worker thread): upload, frame, sgm_check
    static void run_slot(Slot &sl, const Mat &l, const Mat &r) {
        sl.error.clear();
        hipStream_t st = (hipStream_t)sl.stream;
        const size_t w = (size_t)l.cols;
        if (hipSetDevice(sl.device) != hipSuccess ||
            hipMemcpy2DAsync(sl.d_l, w, l.data, (size_t)l.step, w, l.rows, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpy2DAsync(sl.d_r, w, r.data, (size_t)r.step, w, r.rows, hipMemcpyHostToDevice, st) != hipSuccess) {
            sl.error = "uploading the pair failed";
            return;
        }
        int rows = 0, cols = 0;
        sgm_get_size(sl.h, &rows, &cols, nullptr);
        // NULL stream: the handle's own (sl.stream), where the upload went
        if (sgm_process_device(sl.h, sl.d_l, sl.d_r, l.cols, nullptr, nullptr, 0, sl.d_map, cols, nullptr,
                               nullptr) != SGM_OK ||
            sgm_check(sl.h) != SGM_OK)
            sl.error = sgm_last_error(sl.h);
    }

    void release() {
        if (comm_) sgm_comm_destroy(comm_);
        comm_ = nullptr;
        if (d_root_) {
            (void)hipSetDevice(slots_[0].device);
            (void)hipFree(d_root_);
        }
        d_root_ = nullptr;
        for (auto &sl : slots_) {
            if (sl.device >= 0) (void)hipSetDevice(sl.device);
            if (sl.d_l) (void)hipFree(sl.d_l);
            if (sl.d_r) (void)hipFree(sl.d_r);
            if (sl.d_map) (void)hipFree(sl.d_map);
            if (sl.h) sgm_destroy(sl.h);
            sl = Slot();
        }
    }
};

}  // namespace sgm_amd

#endif
