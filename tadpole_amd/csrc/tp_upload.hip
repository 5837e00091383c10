// Host -> device upload of an interaction matrix through a context's pinned
// staging (tp_upload_dev, tp_pipeline's host path).  R/TADpole.R:17 reads the
// matrix into host memory; the pipeline needs it in HBM.  A pageable
// hipMemcpy goes through the runtime's one staging path, which every stream of
// a process shares (C4: 8 chromosomes in flight on one GPU, ~6 GB of float64
// matrices), so the copy runs here: 16 MB blocks through a ring of three
// pinned slots, each block's host pass (nthreads threads) overlapped with the
// previous blocks' DMAs.
//
// Hi-C matrices hold counts.  With `counts`, a block whose every value is an
// exact integer in [0, 65535] (no -0.0, NaN, fraction or larger value) travels
// as 16-bit integers and k_u16_to_f64 widens it on the device -- the same
// doubles bit for bit, a quarter of the PCIe bytes; any other block travels as
// float64.  Nothing is assumed about the matrix: the check is per block, on
// the values themselves.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "tp_common.cuh"
#include "tp_internal.h"

namespace tp {

__global__ void __launch_bounds__(256) k_u16_to_f64(const uint16_t *__restrict__ src, size_t n,
                                                    double *__restrict__ dst) {
    const size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i + 3 < n) {
        const ushort4 v = *(const ushort4 *)(src + i);
        *(double2 *)(dst + i) = make_double2((double)v.x, (double)v.y);
        *(double2 *)(dst + i + 2) = make_double2((double)v.z, (double)v.w);
    } else {
        for (size_t j = i; j < n; ++j) dst[j] = (double)src[j];
    }
}

// values as 16-bit counts, or false (dst then partly written, unused).
// Branch-free per 256-value chunk: t = v clamped to [-1, 65536] (NaN -> -1),
// truncated; the value is a count iff t == v, 0 <= t <= 65535, sign bit clear
static bool pack_u16(const double *src, size_t n, uint16_t *dst) {
    for (size_t i0 = 0; i0 < n; i0 += 256) {
        const size_t i1 = std::min(n, i0 + 256);
        unsigned bad = 0;
        for (size_t i = i0; i < i1; ++i) {
            const double v = src[i];
            uint64_t bits;
            memcpy(&bits, &v, 8);
            const double cl = v > -1.0 ? (v < 65536.0 ? v : 65536.0) : -1.0;   // NaN -> -1
            const int t = (int)cl;
            bad |= (unsigned)((double)t != v) | (unsigned)(t < 0) | (unsigned)(t > 65535) | (unsigned)(bits >> 63);
            dst[i] = (uint16_t)t;
        }
        if (bad) return false;
    }
    return true;
}

// Optionally one upload at a time per device, first come first served
// (concurrent uploads split the PCIe link, ~56 GB/s on the MI355X box, evenly;
// in turn the largest matrix of a genome run, submitted first, gets it whole --
// measured no faster, see t_knob.upload_mode).
struct UploadTurn {
    std::mutex mu;
    std::condition_variable cv;
    unsigned long long next = 0, serving = 0;
};
static UploadTurn g_turn[64];
// knob 43: bit 1 count blocks packed to 16 bits (default), bit 0 uploads in
// turn.  C4 (23 chromosomes, 8 streams, 5 runs each, one box): packed 0.277 s
// median (4.5 % spread), raw 0.299, in turn 0.279-0.284 with runs up to 0.32,
// in turn + packed 0.319 -- staggering the uploads staggers the pipelines
// behind them more than it helps the first one

template <typename F>
static void split_run(size_t n, int th, F f) {   // f(offset, count) over th contiguous parts
    if (th <= 1 || n < ((size_t)1 << 17)) {
        f((size_t)0, n);
        return;
    }
    std::vector<std::thread> ts;
    const size_t part = (n / th + 63) & ~(size_t)63;
    for (int t = 0; t < th; ++t) {
        const size_t o = (size_t)t * part;
        if (o >= n) break;
        ts.emplace_back([=] { f(o, std::min(part, n - o)); });
    }
    for (auto &x : ts) x.join();
}

size_t upload_host(Ctx &c, const void *host, size_t bytes, void *d_dst, int nthreads, bool counts) {
    if (bytes == 0) return 0;
    if (!(t_knob.upload_mode & 2)) counts = false;
    UploadTurn &turn = g_turn[c.device & 63];
    const bool in_turn = (t_knob.upload_mode & 1) != 0;
    unsigned long long ticket = 0;
    if (in_turn) {
        std::unique_lock<std::mutex> lk(turn.mu);
        ticket = turn.next++;
        turn.cv.wait(lk, [&] { return turn.serving == ticket; });
    }
    struct Done {   // the next ticket's turn, also when this upload throws
        UploadTurn &t;
        bool on;
        ~Done() {
            if (!on) return;
            {
                std::lock_guard<std::mutex> lk(t.mu);
                ++t.serving;
            }
            t.cv.notify_all();
        }
    } done{turn, in_turn};
    constexpr int kSlots = 3;
    constexpr size_t kBlock = (size_t)16 << 20;   // bytes of float64 a block
    static_assert(kSlots <= (int)(sizeof(c.ring_ev) / sizeof(c.ring_ev[0])), "Ctx::ring_ev too small");
    if (counts && bytes % sizeof(double)) counts = false;
    for (int q = 0; q < kSlots; ++q)
        if (!c.ring_ev[q]) TP_HIP(hipEventCreateWithFlags(&c.ring_ev[q], hipEventDisableTiming));
    const size_t nb = (bytes + kBlock - 1) / kBlock;
    const size_t slot_bytes = std::min(bytes, kBlock);
    char *ring = (char *)c.pinned(kSlots * slot_bytes);
    uint16_t *dstage = counts ? c.buf[S_UPLD].as<uint16_t>((size_t)kSlots * (kBlock / 8)) : nullptr;
    const int th = std::max(1, std::min(nthreads, 16));
    size_t packed = 0;
    for (size_t b = 0; b < nb; ++b) {
        const int slot = (int)(b % kSlots);
        if (b >= (size_t)kSlots) {   // the slot's previous copy (a 16 MB DMA, < 1 ms)
            hipError_t q;
            while ((q = hipEventQuery(c.ring_ev[slot])) == hipErrorNotReady) std::this_thread::yield();
            TP_HIP(q);
        }
        const size_t off = b * kBlock, len = std::min(kBlock, bytes - off);
        char *pin = ring + (size_t)slot * slot_bytes;
        const char *src = (const char *)host + off;
        bool pk = false;
        if (counts) {   // one packing pass per part; the block is packed if every part is
            const size_t nv = len / sizeof(double);
            std::atomic<bool> ok{true};
            split_run(nv, th, [&](size_t o, size_t n) {
                if (!pack_u16((const double *)src + o, n, (uint16_t *)pin + o)) ok = false;
            });
            pk = ok;
        }
        if (pk) {
            const size_t nv = len / sizeof(double);
            uint16_t *ds = dstage + (size_t)slot * (kBlock / 8);
            TP_HIP(hipMemcpyAsync(ds, pin, nv * sizeof(uint16_t), hipMemcpyHostToDevice, c.cur));
            const unsigned g = (unsigned)((nv + 1023) / 1024);
            hipLaunchKernelGGL(k_u16_to_f64, dim3(g), dim3(256), 0, c.cur, ds, nv, (double *)((char *)d_dst + off));
            TP_HIP(hipGetLastError());
            packed += len;
        } else {
            split_run(len, th, [&](size_t o, size_t n) { memcpy(pin + o, src + o, n); });
            TP_HIP(hipMemcpyAsync((char *)d_dst + off, pin, len, hipMemcpyHostToDevice, c.cur));
        }
        TP_HIP(hipEventRecord(c.ring_ev[slot], c.cur));
    }
    stream_sync(c, c.cur);   // the staging is reused by the next call on this context
    return packed;
}

}  // namespace tp
