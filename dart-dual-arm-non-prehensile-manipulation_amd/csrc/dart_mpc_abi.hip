// dart_mpc_abi.hip -- the C ABI of include/dart_mpc.h (host side).
//
// Owns the device workspace for the host-pointer entry point and the
// per-handle stream; validates arguments the way PMPC.__init__/solve would
// fail (mpc_3d.py:12-138), then launches the batched kernel.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <chrono>
#include <mutex>
#include <vector>
#include <string>

#include "dart_mpc.h"
#include "pmpc_ipm.h"
#include "pmpc_model.h"
#include "wave.h"
#include "rmpc_ipm.h"
#include "lmpc_ipm.h"
#include "lmpc_policy.h"
#include "arm_qp.h"

#include <cmath>

namespace {

// Staging of the host-pointer entries.  The inputs (and the in/out arrays) are packed into pinned
// host memory and reach HBM with ONE DMA copy; the kernel writes its outputs straight into mapped,
// coherent pinned host memory (a few bytes per instance, no copy back); in/out arrays return with
// one more DMA copy.  Against one pageable hipMemcpy per array this removes 5-10 copies per call.
// Capacities grow on demand; a stage is not thread-safe (one per handle, one per device for the
// stateless entries behind a mutex).
struct HostStage {
    char* hin = nullptr;            // pinned: packed inputs | in/out arrays
    char* din = nullptr;            // device mirror of hin
    char* hout = nullptr;           // pinned, mapped, coherent: kernel outputs
    char* dout = nullptr;           // device address of hout
    char* hzc = nullptr;            // pinned, mapped, coherent: zero-copy inputs (read by the kernel over PCIe)
    char* dzc = nullptr;            // device address of hzc
    size_t in_cap = 0, out_cap = 0, zc_cap = 0, in_off = 0, out_off = 0, zc_off = 0, io_first = 0;
    struct Back { void* dst; size_t off, bytes; };
    Back back[8];
    int nback = 0;

    static size_t al(size_t n) { return (n + 255) & ~size_t(255); }
    hipError_t reserve(size_t in_bytes, size_t out_bytes, size_t zc_bytes = 0) {
        hipError_t e = hipSuccess;
        if (zc_bytes > zc_cap) {
            release_zc();
            e = hipHostMalloc((void**)&hzc, zc_bytes, hipHostMallocMapped | hipHostMallocCoherent);
            if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&dzc, hzc, 0);
            if (e != hipSuccess) { release_zc(); return e; }
            zc_cap = zc_bytes;
        }
        if (in_bytes > in_cap) {
            release_in();
            e = hipHostMalloc((void**)&hin, in_bytes, hipHostMallocDefault);
            if (e == hipSuccess) e = hipMalloc((void**)&din, in_bytes);
            if (e != hipSuccess) { release_in(); return e; }
            in_cap = in_bytes;
        }
        if (out_bytes > out_cap) {
            release_out();
            e = hipHostMalloc((void**)&hout, out_bytes, hipHostMallocMapped | hipHostMallocCoherent);
            if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&dout, hout, 0);
            if (e != hipSuccess) { release_out(); return e; }
            out_cap = out_bytes;
        }
        return e;
    }
    void release_in() {
        if (hin) (void)hipHostFree(hin);
        if (din) (void)hipFree(din);
        hin = din = nullptr; in_cap = 0;
    }
    void release_out() {
        if (hout) (void)hipHostFree(hout);
        hout = dout = nullptr; out_cap = 0;
    }
    void release_zc() {
        if (hzc) (void)hipHostFree(hzc);
        hzc = dzc = nullptr; zc_cap = 0;
    }
    void begin() { in_off = out_off = zc_off = 0; nback = 0; io_first = 0; }
    // device-visible pointer of an input the kernel reads straight from mapped host memory: no DMA
    // copy on the call path (for kernels that read their inputs once, at the start)
    template <class T> const T* in_zc(const T* src, size_t n) {
        if (!src) return nullptr;
        const size_t off = zc_off;
        std::memcpy(hzc + off, src, n * sizeof(T));
        zc_off += al(n * sizeof(T));
        return reinterpret_cast<const T*>(dzc + off);
    }
    // device pointer of an input copied from src (n elements); nullptr stays nullptr
    template <class T> const T* in(const T* src, size_t n) {
        if (!src) return nullptr;
        const size_t off = in_off;
        std::memcpy(hin + off, src, n * sizeof(T));
        in_off += al(n * sizeof(T));
        return reinterpret_cast<const T*>(din + off);
    }
    // device pointer of an in/out array (read and updated by the kernel); call these last
    template <class T> T* inout(T* src, size_t n) {
        if (!src) return nullptr;
        if (nback == 0) io_first = in_off;
        const size_t off = in_off;
        in(src, n);
        back[nback++] = Back{src, off, n * sizeof(T)};
        return reinterpret_cast<T*>(din + off);
    }
    // device-visible pointer of an output slot (n elements) in mapped host memory
    template <class T> T* out(size_t n) {
        const size_t off = out_off;
        out_off += al(n * sizeof(T));
        return reinterpret_cast<T*>(dout + off);
    }
    template <class T> const T* host_of(const T* dev_out) const {
        return reinterpret_cast<const T*>(hout + (reinterpret_cast<const char*>(dev_out) - dout));
    }
    hipError_t upload(hipStream_t s) const {
        return in_off ? hipMemcpyAsync(din, hin, in_off, hipMemcpyHostToDevice, s) : hipSuccess;
    }
    hipError_t download_inout(hipStream_t s) const {
        return nback ? hipMemcpyAsync(hin + io_first, din + io_first, in_off - io_first, hipMemcpyDeviceToHost, s)
                     : hipSuccess;
    }
    // after the stream synchronised: in/out arrays back to the caller, then outputs
    void finish_inout() const {
        for (int i = 0; i < nback; ++i) std::memcpy(back[i].dst, hin + back[i].off, back[i].bytes);
    }
    template <class T> void take(T* dst, const T* dev_out, size_t n) const {
        if (dst && dev_out) std::memcpy(dst, host_of(dev_out), n * sizeof(T));
    }
    void release() { release_in(); release_out(); release_zc(); }
};

// stage + stream of the stateless host entries (arm QP, policy step, RLS), one per device
struct DeviceStage {
    std::mutex mu;
    HostStage st;
    hipStream_t stream = nullptr;
};

hipError_t device_stage(DeviceStage** out) {
    static DeviceStage stages[64];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    DeviceStage& d = stages[dev];
    std::lock_guard<std::mutex> g(d.mu);
    if (!d.stream) e = hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking);
    *out = &d;
    return e;
}

}  // namespace

struct dart_mpc_handle {
    dart_mpc_config cfg;
    int device = 0;
    hipStream_t stream = nullptr;
    HostStage st;                  // staging of the host-pointer entries
    std::string err;
    uint32_t seq = 0;              // completion-word sequence of the host-pointer PMPC entry (wraps, skips 0)
    uint32_t* hdone = nullptr;     // PMPC: B_max completion words, mapped host memory (only ever
    uint32_t* ddone = nullptr;     //   hold 0 or sequence numbers of earlier calls) and their device address
    // the host PMPC entry returns once every completion word is visible, possibly before the stream
    // has retired the kernel's last instructions: the next entry on the handle settles that stream
    // first, so a late stream error is reported as the previous call's, not blamed on the new one
    hipStream_t pending = nullptr;
    // resident PMPC server (dart_mpc_serve_start): its own stream, a mailbox, inputs and outputs at
    // fixed mapped addresses for B_serve slots
    struct Server {
        bool wanted = false;               // serve_start called, serve_stop not yet
        bool running = false;
        int B = 0;
        hipStream_t stream = nullptr;
        uint32_t* mbox = nullptr;          // mapped: the 64-bit request word (pmpc_ipm.h PmpcServe)
        uint32_t* dmbox = nullptr;
        unsigned long long idle_ticks = 0;
        double idle_s = 0.0;
        std::chrono::steady_clock::time_point t_post;     // last request posted (or the grid launched)
    } srv;
    // PMPC in-place I/O area (dart_mpc_bind; the resident server's inputs and outputs): mapped,
    // coherent pinned memory for B_max instances at fixed addresses
    struct Io {
        char* hin = nullptr;  char* din = nullptr;      // x0 | ref | prm | w_warm
        char* hout = nullptr; char* dout = nullptr;     // u0 | f | w_out | status | iters
        size_t off_ref = 0, off_prm = 0, off_ww = 0, off_f = 0, off_wo = 0, off_st = 0, off_it = 0;
    } io;
    // Serialises the entries on this handle: the host-pointer entries share the pinned staging
    // buffers and the handle's stream, and every entry may write err.  Concurrent callers (the
    // reference runs controllers on background threads, RMPC/dev_dual/controller/convimp.py:435)
    // are safe but take turns; one handle per thread runs them side by side.
    std::recursive_mutex mu;     // recursive: the host entries call their _dev twins
    // LMPC: hand-off areas of the instances that enter IPOPT's restoration phases (lmpc_ipm.hip,
    // [B][64][16] doubles), one per launch stream -- launches in flight on different streams never share
    // one -- grown on demand by stream-ordered allocation (the old area is freed behind its last use on
    // that stream: no device-wide synchronisation, nothing else waits)
    struct RestoArea {
        hipStream_t s;
        double* buf;
        size_t cap;
        int xcd;                   // XCD of the stream's small batches (round robin over the streams)
    };
    std::vector<RestoArea> resto;
    unsigned xcd_next = 0;
};

namespace {

int fail(dart_mpc_handle* h, int code, const char* what, hipError_t e = hipSuccess) {
    if (h) {
        char buf[256];
        if (e != hipSuccess) std::snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
        else std::snprintf(buf, sizeof buf, "%s", what);
        h->err = buf;
    }
    return code;
}

#define HIPCHK(h, call, what)                                          \
    do {                                                               \
        hipError_t e_ = (call);                                        \
        if (e_ != hipSuccess) return fail((h), DART_MPC_EHIP, (what), e_); \
    } while (0)

int check_cfg(const dart_mpc_config* c) {
    if (!c) return 0;
    if (c->variant != DART_MPC_PMPC && c->variant != DART_MPC_RMPC && c->variant != DART_MPC_LMPC) return 0;
    if (c->N < 1 || c->N > 63) return 0;
    if (!(c->Ts > 0.0) || !(c->tol > 0.0) || !(c->gravity == c->gravity) || c->max_iter < 1 || c->B_max < 1) return 0;
    if (c->acceptable_iter < 0 || (c->acceptable_iter > 0 && !(c->acceptable_tol > 0.0))) return 0;
    if (c->max_soc < 0 || c->max_soc > 8) return 0;
    if (c->pmpc_path != 0 && c->pmpc_path != 1) return 0;
    if (!(c->constr_mult_init_max >= 0.0)) return 0;
    if (!(c->max_cpu_time >= 0.0) || c->max_cpu_time > 1e9) return 0;
    return 1;
}

void server_release(dart_mpc_handle* h) {
    auto& v = h->srv;
    if (v.mbox) (void)hipHostFree(v.mbox);
    if (v.stream) (void)hipStreamDestroy(v.stream);
    v = dart_mpc_handle::Server{};
}

void io_release(dart_mpc_handle* h) {
    auto& o = h->io;
    if (o.hin) (void)hipHostFree(o.hin);
    if (o.hout) (void)hipHostFree(o.hout);
    o = dart_mpc_handle::Io{};
}

// the in-place I/O area for B_max instances (allocated once)
hipError_t ensure_io(dart_mpc_handle* h) {
    auto& o = h->io;
    if (o.hin) return hipSuccess;
    const size_t nw = (size_t)dart_mpc_nw(h->cfg.N), Bm = (size_t)h->cfg.B_max;
    auto al = [](size_t n) { return (n + 255) & ~size_t(255); };
    o.off_ref = al(sizeof(double) * 6 * Bm); o.off_prm = 2 * o.off_ref; o.off_ww = 3 * o.off_ref;
    const size_t in_bytes = o.off_ww + al(sizeof(double) * nw * Bm);
    o.off_f = al(sizeof(double) * 2 * Bm); o.off_wo = o.off_f + al(sizeof(double) * Bm);
    o.off_st = o.off_wo + al(sizeof(double) * nw * Bm); o.off_it = o.off_st + al(sizeof(int32_t) * Bm);
    const size_t out_bytes = o.off_it + al(sizeof(int32_t) * Bm);
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    hipError_t e = hipHostMalloc((void**)&o.hin, in_bytes, fl);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&o.din, o.hin, 0);
    if (e == hipSuccess) e = hipHostMalloc((void**)&o.hout, out_bytes, fl);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&o.dout, o.hout, 0);
    if (e != hipSuccess) { io_release(h); return e; }
    std::memset(o.hin, 0, in_bytes);
    std::memset(o.hout, 0, out_bytes);
    return hipSuccess;
}

// IPOPT's restoration phases for PMPC launches of this handle (pmpc_resto.h: IPOPT's path, N <= 31);
// `mode` 1 for launches whose restoration runs on the device without the host (the launcher runs it in the
// solving wave for B <= 32, else queues pmpc_resto_kernel behind the solve), 2 for launches whose handed-over
// instances the host sees in their completion words (it launches the kernel only then: host_resto)
int pmpc_resto_mode(const dart_mpc_handle* h, int mode) {
    return (h->cfg.restoration && h->cfg.pmpc_path == 0 && h->cfg.N <= 31) ? mode : 0;
}

// IPOPT's soft restoration phase in the register kernel: with the restoration phases on, on IPOPT's path, at every N
int pmpc_soft(const dart_mpc_handle* h) { return (h->cfg.restoration && h->cfg.pmpc_path == 0) ? 1 : 0; }

// the mode of a host-entry launch of B instances: in the solving wave (small batches), else host-driven
int host_resto_mode(const dart_mpc_handle* h, int B) { return pmpc_resto_mode(h, B <= 32 ? 1 : 2); }

// After the completion words of a host-driven (mode 2) launch: pmpc_resto_kernel for the handed-over
// instances (status kPmNeedResto, read from mapped host memory), only if there is one -- no restoration
// dispatch follows a batch that needs none
int host_resto(dart_mpc_handle* h, dartmpc::PmpcArgs a, const int32_t* host_status, hipStream_t s) {
    if (a.resto != 2) return DART_MPC_OK;
    bool any = false;
    for (int b = 0; b < a.B && !any; ++b)
        any = __atomic_load_n(host_status + b, __ATOMIC_ACQUIRE) == dartmpc::kPmNeedResto;
    if (!any) return DART_MPC_OK;
    a.done = nullptr;
    HIPCHK(h, dartmpc_launch_pmpc_resto(&a, s), "restoration kernel launch");
    HIPCHK(h, hipStreamSynchronize(s), "restoration kernel");
    return DART_MPC_OK;
}

int stream_state(dart_mpc_handle* h, int B, hipStream_t s, double** out, int* xcd);

// the restoration hand-off area of a PMPC launch of B instances on stream s (when the launch can hand over)
int pmpc_resto_buf(dart_mpc_handle* h, int B, hipStream_t s, dartmpc::PmpcArgs& a) {
    a.resto_buf = nullptr;
    // Resuming from the register kernel's failed iteration is opt-in (DART_PMPC_RESUME=1): the register kernel's
    // iterate differs from the sequential (oracle-ordered) arithmetic by rounding, and the restoration phase
    // turns that into different iteration counts on ~19 % of the restored instances (the same statuses, u0
    // within 1.3e-11; tools/pmpc_resume_check.py, profiles/r05/pmpc_resume.txt).  By default the restoration
    // solve starts over on the LDS engine and takes the oracle's iterations exactly.
    static const bool resume = [] {
        const char* e = getenv("DART_PMPC_RESUME");
        return e && e[0] == '1';
    }();
    if (!a.resto || !resume) return DART_MPC_OK;
    int xcd = 0;
    return stream_state(h, B, s, &a.resto_buf, &xcd);
}

// kernel arguments reading / writing the I/O area
dartmpc::PmpcArgs io_args(dart_mpc_handle* h, int B, bool ww, bool wo, int resto_mode = 1) {
    const auto& o = h->io;
    dartmpc::PmpcArgs a;
    a.B = B; a.N = h->cfg.N; a.Ts = h->cfg.Ts; a.tol = h->cfg.tol; a.max_iter = h->cfg.max_iter; a.g = h->cfg.gravity;
    a.max_soc = h->cfg.max_soc; a.reduced = h->cfg.pmpc_path; a.mult_init_max = h->cfg.constr_mult_init_max;
    a.x0 = (const double*)o.din; a.ref = (const double*)(o.din + o.off_ref); a.prm = (const double*)(o.din + o.off_prm);
    a.w_warm = ww ? (const double*)(o.din + o.off_ww) : nullptr;
    a.u0 = (double*)o.dout; a.f = (double*)(o.dout + o.off_f); a.w_out = wo ? (double*)(o.dout + o.off_wo) : nullptr;
    a.status = (int32_t*)(o.dout + o.off_st); a.iters = (int32_t*)(o.dout + o.off_it);
    a.done = h->ddone; a.seq = h->seq;
    a.resto = pmpc_resto_mode(h, resto_mode);
    a.soft = pmpc_soft(h);
    a.resto_buf = nullptr;        // (the caller sets it for its stream: pmpc_resto_buf)
    return a;
}

// (re)launch the resident grid; it takes every request with a sequence other than `seen`
hipError_t server_launch(dart_mpc_handle* h, uint32_t seen) {
    auto& v = h->srv;
    dartmpc::PmpcArgs a = io_args(h, v.B, true, true, 2);  // the flags of each request select w_warm / w_out
    a.seq = seen;
    if (pmpc_resto_buf(h, v.B, v.stream, a) != DART_MPC_OK) return hipErrorOutOfMemory;
    dartmpc::PmpcServe sv{v.dmbox, v.idle_ticks};
    const hipError_t e = dartmpc_launch_pmpc_serve(&a, &sv, v.stream);
    v.running = e == hipSuccess;
    v.t_post = std::chrono::steady_clock::now();
    return e;
}

// stop the resident server (if any) and wait until its grid has drained
int server_stop(dart_mpc_handle* h) {
    auto& v = h->srv;
    if (!v.stream) return DART_MPC_OK;
    __atomic_store_n((unsigned long long*)v.mbox, (unsigned long long)v.mbox[0] | (1ull << 56), __ATOMIC_RELEASE);
    const hipError_t e = hipStreamSynchronize(v.stream);
    v.running = false;
    server_release(h);
    return e == hipSuccess ? DART_MPC_OK : fail(h, DART_MPC_EHIP, "resident server", e);
}

// The per-stream state of PMPC / LMPC launches on stream s: the restoration hand-off area for B instances
// (device memory, stream-ordered growth: see dart_mpc_handle::resto; PMPC pmpc_model.h kPmHo doubles per
// instance, LMPC 64 x 16) and the XCD that a small LMPC batch's working blocks take -- streams get XCDs round
// robin, so that batches in flight on different streams of a handle run side by side on different XCDs instead
// of queueing for the CUs of one
int stream_state(dart_mpc_handle* h, int B, hipStream_t s, double** out, int* xcd) {
    *out = nullptr;
    // per instance: PMPC's hand-off state, LMPC's hand-off state (N > 31: and the two-wave build's second-order-
    // correction and restoration state, needed with or without the restoration phases), RMPC's two-wave
    // restoration state
    const bool wg2 = h->cfg.N > 31 || dartmpc::force_wg2();
    const size_t per = h->cfg.variant == DART_MPC_PMPC   ? (size_t)dartmpc::kPmHo
                       : h->cfg.variant == DART_MPC_RMPC ? (dartmpc_rmpc_wg2_resto_bytes() + 7) / 8
                       : wg2                             ? dartmpc_lmpc_wg2_area_doubles()
                                                         : (size_t)64 * 16;
    const size_t need = (h->cfg.restoration || (wg2 && h->cfg.variant == DART_MPC_LMPC)) ? (size_t)B * per : 0;
    dart_mpc_handle::RestoArea* r = nullptr;
    for (auto& e : h->resto)
        if (e.s == s) r = &e;
    if (!r) {
        // at most kMaxRestoAreas streams keep an area: the least recently used one is freed (a caller that makes
        // a new stream per call does not grow device memory without bound).  Its stream may be gone by now, so the
        // area is freed with hipFree, which waits for the device's outstanding work first (this rare path only).
        constexpr size_t kMaxRestoAreas = 8;
        if (h->resto.size() >= kMaxRestoAreas) {
            // (never the resident server's: its grid may hand an instance over into it at any time)
            size_t v = 0;
            while (v + 1 < h->resto.size() && h->srv.stream && h->resto[v].s == h->srv.stream) ++v;
            dart_mpc_handle::RestoArea old = h->resto[v];
            h->resto.erase(h->resto.begin() + v);
            if (old.buf) HIPCHK(h, hipFree(old.buf), "hipFree (restoration hand-off)");
        }
        h->resto.push_back({s, nullptr, 0, (int)(h->xcd_next++ & 7u)});
        r = &h->resto.back();
    } else if (r != &h->resto.back()) {     // most recently used last
        dart_mpc_handle::RestoArea cur = *r;
        h->resto.erase(h->resto.begin() + (r - h->resto.data()));
        h->resto.push_back(cur);
        r = &h->resto.back();
    }
    if (need > r->cap) {
        if (r->buf) HIPCHK(h, hipFreeAsync(r->buf, s), "hipFreeAsync (restoration hand-off)");
        r->buf = nullptr; r->cap = 0;
        HIPCHK(h, hipMallocAsync((void**)&r->buf, need * sizeof(double), s), "hipMallocAsync (restoration hand-off)");
        r->cap = need;
    }
    *out = r->buf;
    *xcd = r->xcd;
    return DART_MPC_OK;
}

int settle_pending(dart_mpc_handle* h) {
    if (!h->pending) return DART_MPC_OK;
    hipStream_t s = h->pending;
    h->pending = nullptr;
    hipError_t e = hipStreamQuery(s);
    if (e == hipErrorNotReady) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fail(h, DART_MPC_EHIP, "previous PMPC call's stream", e);
    return DART_MPC_OK;
}

int launch(dart_mpc_handle* h, int B, const double* x0, const double* ref, const double* prm, const double* w_warm,
           double* u0, double* f, double* w_out, int32_t* status, int32_t* iters, hipStream_t s) {
    dartmpc::PmpcArgs a;
    a.B = B; a.N = h->cfg.N; a.Ts = h->cfg.Ts; a.tol = h->cfg.tol; a.max_iter = h->cfg.max_iter; a.g = h->cfg.gravity;
    a.max_soc = h->cfg.max_soc; a.reduced = h->cfg.pmpc_path;
    a.mult_init_max = h->cfg.constr_mult_init_max;
    a.x0 = x0; a.ref = ref; a.prm = prm; a.w_warm = w_warm;
    a.u0 = u0; a.f = f; a.w_out = w_out; a.status = status; a.iters = iters;
    a.done = nullptr; a.seq = 0;
    a.resto = pmpc_resto_mode(h, 1);
    a.soft = pmpc_soft(h);
    if (int rc = pmpc_resto_buf(h, B, s, a)) return rc;
    HIPCHK(h, dartmpc_launch_pmpc(&a, s), "kernel launch");
    return DART_MPC_OK;
}

// Wait for the B completion words of a host-pointer PMPC launch (mapped host memory, written last by
// every instance with a system-scope release).  Spinning on them returns as soon as the last store
// lands, without the stream-completion round trip; the stream is queried now and then, and if it is
// done (or failed) without every word set, the stream's own status decides.
int wait_done(dart_mpc_handle* h, hipStream_t s, const volatile uint32_t* done, int B, uint32_t seq) {
    for (unsigned n = 1;; ++n) {
        int b = 0;
        while (b < B && __atomic_load_n(done + b, __ATOMIC_ACQUIRE) == seq) ++b;
        if (b == B) return DART_MPC_OK;
        if ((n & 255) == 0 && hipStreamQuery(s) != hipErrorNotReady) break;
        __builtin_ia32_pause();
    }
    HIPCHK(h, hipStreamSynchronize(s), "hipStreamSynchronize");
    for (int b = 0; b < B; ++b)
        if (__atomic_load_n(done + b, __ATOMIC_ACQUIRE) != seq) return fail(h, DART_MPC_EHIP, "kernel did not complete");
    return DART_MPC_OK;
}

// the next completion-word sequence of the handle (wraps, skipping 0; on a wrap every word is cleared so that
// no stale one can match: the words only ever hold 0 or sequences of earlier requests)
uint32_t next_seq(dart_mpc_handle* h) {
    if (++h->seq == 0) {
        std::memset(h->hdone, 0, sizeof(uint32_t) * h->cfg.B_max);
        h->seq = 1;
    }
    return h->seq;
}

// A served request's instances that the resident grid handed over (status kPmNeedResto: IPOPT's restoration
// phases): the grid is drained (its waves hold the SIMDs while they wait for requests) and pmpc_resto_kernel
// runs over the I/O area on the server's stream; the next request relaunches the grid.
int served_resto(dart_mpc_handle* h, int B, bool ww, bool wo) {
    auto& v = h->srv;
    const int32_t* st = (const int32_t*)(h->io.hout + h->io.off_st);
    bool any = false;
    for (int b = 0; b < B && !any; ++b) any = __atomic_load_n(st + b, __ATOMIC_ACQUIRE) == dartmpc::kPmNeedResto;
    if (!any) return DART_MPC_OK;
    __atomic_store_n((unsigned long long*)v.mbox, (unsigned long long)v.mbox[0] | (1ull << 56), __ATOMIC_RELEASE);
    v.running = false;
    HIPCHK(h, hipStreamSynchronize(v.stream), "resident server");
    dartmpc::PmpcArgs a = io_args(h, B, ww, wo, 1);
    a.done = nullptr;
    if (int rc = pmpc_resto_buf(h, v.B, v.stream, a)) return rc;      // the area the grid handed over into
    HIPCHK(h, dartmpc_launch_pmpc_resto(&a, v.stream), "restoration kernel launch");
    HIPCHK(h, hipStreamSynchronize(v.stream), "restoration kernel");
    return DART_MPC_OK;
}

// post a request to the resident server (inputs already in the I/O area) and wait for its B
// completion words; a grid that drained meanwhile (idle timeout) is relaunched and takes the request
int served_request(dart_mpc_handle* h, int B, bool ww, bool wo) {
    auto& v = h->srv;
    // Every wave leaves idle_timeout after the last request it saw, each on its own clock, so near the end of
    // an idle period part of the grid may have left while the rest still waits (and a request posted then
    // would reset the waiting waves' timers and wait out a whole idle period for the missing ones).  The host
    // knows when it posted last: from 90 % of the idle timeout on, it drains the grid itself (stop word) and
    // relaunches it before posting.  Before that point no wave can have left (each wave's last request is no
    // older than the host's last post).
    const double since = std::chrono::duration<double>(std::chrono::steady_clock::now() - v.t_post).count();
    // The margin between this check and a wave's own timeout is 10 % of the timeout + 2 ms, capped at half the
    // timeout (so that short timeouts still serve from the grid), but never below 2 ms: a host stall between the
    // check and the post longer than the margin could let part of the grid leave, and the request would then
    // wait out a further idle period.  Timeouts of 4 ms and less therefore pre-drain (relaunch) whenever more
    // than idle - 2 ms has passed: a latency cost, never a stall.
    const double margin = std::fmax(0.002, std::fmin(0.1 * v.idle_s + 0.002, 0.5 * v.idle_s));
    if (v.running && since > v.idle_s - margin) {
        __atomic_store_n((unsigned long long*)v.mbox, (unsigned long long)v.mbox[0] | (1ull << 56), __ATOMIC_RELEASE);
        v.running = false;
    }
    if (!v.running || hipStreamQuery(v.stream) != hipErrorNotReady) {     // drained (idle timeout or stop)
        v.running = false;
        HIPCHK(h, hipStreamSynchronize(v.stream), "resident server");
        __atomic_store_n((unsigned long long*)v.mbox, (unsigned long long)h->seq, __ATOMIC_RELEASE);   // no stop, no request
        HIPCHK(h, server_launch(h, h->seq), "resident server relaunch");
    }
    const uint32_t sq = next_seq(h);
    const unsigned long long fl = (ww ? 1ull : 0ull) | (wo ? 2ull : 0ull);
    __atomic_store_n((unsigned long long*)v.mbox, (unsigned long long)sq | ((unsigned long long)B << 32) | (fl << 48),
                     __ATOMIC_RELEASE);
    v.t_post = std::chrono::steady_clock::now();
    for (unsigned n = 1;; ++n) {
        int bb = 0;
        while (bb < B && __atomic_load_n(h->hdone + bb, __ATOMIC_ACQUIRE) == sq) ++bb;
        if (bb == B) return served_resto(h, B, ww, wo);
        if ((n & 1023) == 0 && hipStreamQuery(v.stream) != hipErrorNotReady) {
            bb = 0;
            while (bb < B && __atomic_load_n(h->hdone + bb, __ATOMIC_ACQUIRE) == sq) ++bb;
            if (bb == B) return served_resto(h, B, ww, wo);
            v.running = false;
            HIPCHK(h, hipStreamSynchronize(v.stream), "resident server");
            // the grid drained before it saw the request: relaunch with the request already posted
            HIPCHK(h, server_launch(h, sq - 1), "resident server relaunch");
        }
        __builtin_ia32_pause();
    }
}

// one launch over the I/O area (no resident server), completion words as the host entry
int bound_launch(dart_mpc_handle* h, int B, bool ww, bool wo) {
    next_seq(h);
    dartmpc::PmpcArgs a = io_args(h, B, ww, wo, B <= 32 ? 1 : 2);
    if (int rc = pmpc_resto_buf(h, B, h->stream, a)) return rc;
    HIPCHK(h, dartmpc_launch_pmpc(&a, h->stream), "kernel launch");
    int rc = wait_done(h, h->stream, h->hdone, B, a.seq);
    if (rc == DART_MPC_OK) rc = host_resto(h, a, (const int32_t*)(h->io.hout + h->io.off_st), h->stream);
    if (rc == DART_MPC_OK) h->pending = h->stream;
    return rc;
}

}  // namespace

extern "C" {

void dart_mpc_config_default(dart_mpc_config* c) {
    if (!c) return;
    c->variant = DART_MPC_PMPC;
    c->N = 20;
    c->Ts = 0.002;
    c->tol = 1e-8;
    c->max_iter = 3000;
    c->B_max = 1024;
    c->gravity = -9.81;
    c->acceptable_tol = 1e-6;      // IPOPT defaults
    c->acceptable_iter = 15;
    c->max_soc = 4;
    c->pmpc_path = 0;
    c->constr_mult_init_max = 1000.0;
    c->restoration = 1;
    c->max_cpu_time = 0.05;         // rlmpc2.py:485
}

int dart_mpc_nw(int N) { return 6 * (N + 1) + 2 * N; }

int dart_rmpc_nw(int N) { return 4 * (N + 1) + 2 * N; }

int dart_lmpc_nw(int N) { return 8 * (N + 1) + 2 * N; }

int dart_mpc_abi_version(void) { return DART_MPC_ABI_VERSION; }
#ifndef DART_BUILD_ID
#define DART_BUILD_ID "unknown"
#endif
const char* dart_mpc_build_id(void) { return DART_BUILD_ID; }
const char* dart_mpc_build_flavor(void) {
#if defined(DART_STAMPS)
    return "stamps";
#elif defined(DART_RESTO_TRACE)
    return "trace";
#else
    return "";
#endif
}

int dart_mpc_create(const dart_mpc_config* cfg, int device, dart_mpc_handle** out) {
    if (!out || !check_cfg(cfg)) return DART_MPC_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return DART_MPC_ENODEV;
    dart_mpc_handle* h = new dart_mpc_handle();
    h->cfg = *cfg;
    h->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    // staging for B_max instances: inputs (+ in/out arrays) and outputs, 256-byte aligned per array
    const size_t B = (size_t)cfg->B_max, A = 8 * 256;
    size_t nin = 0, nout = 0;
    if (cfg->variant == DART_MPC_LMPC) {
        const size_t nw = (size_t)dart_lmpc_nw(cfg->N);
        nin = B * (8 + 2 + dartmpc::LM_NPV + 8 + dartmpc::LM_NPRM + nw);
        nout = B * (2 + 1 + nw + 1);
    } else if (cfg->variant == DART_MPC_RMPC) {
        const size_t nw = (size_t)dart_rmpc_nw(cfg->N);
        nin = B * (4 + 2 + 14 + 98 + 7 + 2 + 4 * (cfg->N + 1) + 10 + nw);
        nout = B * (2 + 1 + nw + 1);
    } else {
        const size_t nw = (size_t)dart_mpc_nw(cfg->N);
        nin = B * (6 + 6 + 6 + nw);
        nout = B * (2 + 1 + nw + 1);
    }
    // PMPC reads its inputs zero-copy (dart_mpc_solve_batch): their pinned buffer is the mapped one
    const bool zc = cfg->variant == DART_MPC_PMPC;
    if (e == hipSuccess)
        e = h->st.reserve(zc ? A : nin * sizeof(double) + A, nout * sizeof(double) + A, zc ? nin * sizeof(double) + A : 0);
    if (e == hipSuccess && zc) {
        e = hipHostMalloc((void**)&h->hdone, sizeof(uint32_t) * B, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) {
            std::memset(h->hdone, 0, sizeof(uint32_t) * B);
            e = hipHostGetDevicePointer((void**)&h->ddone, h->hdone, 0);
        }
    }
    if (e != hipSuccess) {
        dart_mpc_destroy(h);
        return DART_MPC_EHIP;
    }
    *out = h;
    return DART_MPC_OK;
}

int dart_mpc_solve_batch_dev(dart_mpc_handle* h, int B, const double* x0, const double* ref, const double* prm,
                             const double* w_warm, double* u0, double* f, double* w_out, int32_t* status,
                             int32_t* iters, void* stream) {
    if (!h) return DART_MPC_EINVAL;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    if (h->cfg.variant != DART_MPC_PMPC) return fail(h, DART_MPC_EINVAL, "handle is not a PMPC handle");
    if (B < 0 || (B > 0 && (!x0 || !ref || !prm || !u0 || !f || !status || !iters)))
        return fail(h, DART_MPC_EINVAL, "null pointer or negative batch");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    if (int rc = settle_pending(h)) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    return launch(h, B, x0, ref, prm, w_warm, u0, f, w_out, status, iters, s);
}

int dart_mpc_solve_batch(dart_mpc_handle* h, int B, const double* x0, const double* ref, const double* prm,
                         const double* w_warm, double* u0, double* f, double* w_out, int32_t* status,
                         int32_t* iters, void* stream) {
    if (!h) return DART_MPC_EINVAL;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    if (h->cfg.variant != DART_MPC_PMPC) return fail(h, DART_MPC_EINVAL, "handle is not a PMPC handle");
    if (B < 0 || (B > 0 && (!x0 || !ref || !prm || !u0 || !f || !status || !iters)))
        return fail(h, DART_MPC_EINVAL, "null pointer or negative batch");
    if (B > h->cfg.B_max) return fail(h, DART_MPC_EINVAL, "batch larger than B_max");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    if (int rc = settle_pending(h)) return rc;
    const size_t nw = (size_t)dart_mpc_nw(h->cfg.N);
    if (h->srv.wanted && B <= h->srv.B && !stream) {
        // resident server: inputs into the I/O area, the request posted by the request word
        const auto& o = h->io;
        std::memcpy(o.hin, x0, sizeof(double) * 6 * B);
        std::memcpy(o.hin + o.off_ref, ref, sizeof(double) * 6 * B);
        std::memcpy(o.hin + o.off_prm, prm, sizeof(double) * 6 * B);
        if (w_warm) std::memcpy(o.hin + o.off_ww, w_warm, sizeof(double) * nw * B);
        if (int rc = served_request(h, B, w_warm != nullptr, w_out != nullptr)) return rc;
        std::memcpy(u0, o.hout, sizeof(double) * 2 * B);
        std::memcpy(f, o.hout + o.off_f, sizeof(double) * B);
        if (w_out) std::memcpy(w_out, o.hout + o.off_wo, sizeof(double) * nw * B);
        std::memcpy(status, o.hout + o.off_st, sizeof(int32_t) * B);
        std::memcpy(iters, o.hout + o.off_it, sizeof(int32_t) * B);
        return DART_MPC_OK;
    }
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;

    HostStage& S = h->st;
    S.begin();
    // the PMPC kernel reads x0 / ref / prm / w_warm once, at its start: zero-copy from mapped host
    // memory instead of a DMA copy on the call path
    const double* d_x0 = S.in_zc(x0, 6 * B);
    const double* d_ref = S.in_zc(ref, 6 * B);
    const double* d_prm = S.in_zc(prm, 6 * B);
    const double* d_ww = S.in_zc(w_warm, nw * B);
    double* d_u0 = S.out<double>(2 * B);
    double* d_f = S.out<double>(B);
    double* d_wo = w_out ? S.out<double>(nw * B) : nullptr;
    int32_t* d_st = S.out<int32_t>(B);
    int32_t* d_it = S.out<int32_t>(B);
    uint32_t* d_done = h->ddone;
    HIPCHK(h, S.upload(s), "copy inputs");
    dartmpc::PmpcArgs a;
    a.B = B; a.N = h->cfg.N; a.Ts = h->cfg.Ts; a.tol = h->cfg.tol; a.max_iter = h->cfg.max_iter; a.g = h->cfg.gravity;
    a.max_soc = h->cfg.max_soc; a.reduced = h->cfg.pmpc_path;
    a.mult_init_max = h->cfg.constr_mult_init_max;
    a.x0 = d_x0; a.ref = d_ref; a.prm = d_prm; a.w_warm = d_ww;
    a.u0 = d_u0; a.f = d_f; a.w_out = d_wo; a.status = d_st; a.iters = d_it;
    a.done = d_done; a.seq = next_seq(h);
    a.resto = host_resto_mode(h, B);
    a.soft = pmpc_soft(h);
    if (int rc = pmpc_resto_buf(h, B, s, a)) return rc;
    HIPCHK(h, dartmpc_launch_pmpc(&a, s), "kernel launch");
    int rc = wait_done(h, s, h->hdone, B, a.seq);
    if (rc == DART_MPC_OK) rc = host_resto(h, a, S.host_of(d_st), s);
    if (rc) return rc;
    h->pending = s;
    S.take(u0, d_u0, 2 * B); S.take(f, d_f, B); S.take(w_out, d_wo, nw * B);
    S.take(status, d_st, B); S.take(iters, d_it, B);
    return DART_MPC_OK;
}

int dart_rmpc_solve_batch_dev(dart_mpc_handle* h, int B, const double* x0, const double* u_prev, double* theta,
                              double* rls_P, const double* rls_phi, const double* rls_y, double rls_lambda,
                              const double* Rref, const double* prm, const double* w_warm, double* u0, double* f,
                              double* w_out, int32_t* status, int32_t* iters, void* stream) {
    if (!h) return DART_MPC_EINVAL;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    if (h->cfg.variant != DART_MPC_RMPC) return fail(h, DART_MPC_EINVAL, "handle is not an RMPC handle");
    if (B < 0 || (B > 0 && (!x0 || !u_prev || !theta || !Rref || !prm || !u0 || !f || !status || !iters)))
        return fail(h, DART_MPC_EINVAL, "null pointer or negative batch");
    if (rls_P && (!rls_phi || !rls_y || !(rls_lambda > 0.0))) return fail(h, DART_MPC_EINVAL, "RLS inputs incomplete");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    dartmpc::RmpcArgs a;
    a.B = B; a.N = h->cfg.N; a.Ts = h->cfg.Ts; a.tol = h->cfg.tol; a.g = h->cfg.gravity; a.max_iter = h->cfg.max_iter; a.mult_init_max = h->cfg.constr_mult_init_max;
    a.resto = h->cfg.restoration; a.max_soc = h->cfg.max_soc;
    a.x0 = x0; a.u_prev = u_prev; a.theta = theta; a.rls_P = rls_P; a.rls_phi = rls_phi; a.rls_y = rls_y;
    a.rls_lambda = rls_lambda; a.Rref = Rref; a.prm = prm; a.w_warm = w_warm;
    a.u0 = u0; a.f = f; a.w_out = w_out; a.status = status; a.iters = iters;
    a.resto_buf = nullptr;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    if ((a.N > 31 || dartmpc::force_wg2()) && a.resto) {      // the two-wave build's restoration state, one area per stream
        int xcd = 0;
        if (int rc = stream_state(h, B, s, &a.resto_buf, &xcd)) return rc;
    }
    HIPCHK(h, dartmpc_launch_rmpc(&a, s), "kernel launch");
    return DART_MPC_OK;
}

int dart_rmpc_solve_batch(dart_mpc_handle* h, int B, const double* x0, const double* u_prev, double* theta,
                          double* rls_P, const double* rls_phi, const double* rls_y, double rls_lambda,
                          const double* Rref, const double* prm, const double* w_warm, double* u0, double* f,
                          double* w_out, int32_t* status, int32_t* iters, void* stream) {
    if (!h) return DART_MPC_EINVAL;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    if (h->cfg.variant != DART_MPC_RMPC) return fail(h, DART_MPC_EINVAL, "handle is not an RMPC handle");
    if (B < 0 || (B > 0 && (!x0 || !u_prev || !theta || !Rref || !prm || !u0 || !f || !status || !iters)))
        return fail(h, DART_MPC_EINVAL, "null pointer or negative batch");
    if (rls_P && (!rls_phi || !rls_y || !(rls_lambda > 0.0))) return fail(h, DART_MPC_EINVAL, "RLS inputs incomplete");
    if (B > h->cfg.B_max) return fail(h, DART_MPC_EINVAL, "batch larger than B_max");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    const size_t N = (size_t)h->cfg.N, nw = (size_t)dart_rmpc_nw(h->cfg.N);
    HostStage& S = h->st;
    S.begin();
    const double* d_x0 = S.in(x0, 4 * B);
    const double* d_up = S.in(u_prev, 2 * B);
    const double* d_phi = rls_P ? S.in(rls_phi, 7 * B) : nullptr;
    const double* d_y = rls_P ? S.in(rls_y, 2 * B) : nullptr;
    const double* d_R = S.in(Rref, 4 * (N + 1) * B);
    const double* d_prm = S.in(prm, 10 * B);
    const double* d_ww = S.in(w_warm, nw * B);
    // theta is updated in place only when the RLS step is fused
    double* d_th = rls_P ? S.inout(theta, 14 * B) : const_cast<double*>(S.in(theta, 14 * B));
    double* d_P = rls_P ? S.inout(rls_P, 98 * B) : nullptr;
    double* d_u0 = S.out<double>(2 * B);
    double* d_f = S.out<double>(B);
    double* d_wo = w_out ? S.out<double>(nw * B) : nullptr;
    int32_t* d_st = S.out<int32_t>(B);
    int32_t* d_it = S.out<int32_t>(B);
    HIPCHK(h, S.upload(s), "copy inputs");
    int rc = dart_rmpc_solve_batch_dev(h, B, d_x0, d_up, d_th, d_P, d_phi, d_y, rls_lambda, d_R, d_prm, d_ww, d_u0, d_f,
                                       d_wo, d_st, d_it, s);
    if (rc) return rc;
    HIPCHK(h, S.download_inout(s), "copy theta / rls_P");
    HIPCHK(h, hipStreamSynchronize(s), "hipStreamSynchronize");
    S.finish_inout();
    S.take(u0, d_u0, 2 * B); S.take(f, d_f, B); S.take(w_out, d_wo, nw * B);
    S.take(status, d_st, B); S.take(iters, d_it, B);
    return DART_MPC_OK;
}

int dart_lmpc_solve_batch_dev(dart_mpc_handle* h, int B, const double* state, const double* u_prev,
                              const double* pvec, const double* target, const double* prm, const double* w_warm,
                              double* u0, double* f, double* w_out, int32_t* status, int32_t* iters, void* stream) {
    if (!h) return DART_MPC_EINVAL;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    if (h->cfg.variant != DART_MPC_LMPC) return fail(h, DART_MPC_EINVAL, "handle is not an LMPC handle");
    if (B < 0 || (B > 0 && (!state || !u_prev || !pvec || !target || !prm || !u0 || !f || !status || !iters)))
        return fail(h, DART_MPC_EINVAL, "null pointer or negative batch");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    dartmpc::LmpcArgs a;
    a.B = B; a.N = h->cfg.N; a.Ts = h->cfg.Ts; a.tol = h->cfg.tol; a.max_iter = h->cfg.max_iter;
    a.acc_tol = h->cfg.acceptable_tol; a.acc_iter = h->cfg.acceptable_iter; a.max_soc = h->cfg.max_soc; a.mult_init_max = h->cfg.constr_mult_init_max;
    a.resto = h->cfg.restoration;
    a.max_ticks = (long long)(h->cfg.max_cpu_time * 1e8);     // s_memrealtime: 100 MHz
    if (int rc = stream_state(h, B, stream ? (hipStream_t)stream : h->stream, &a.resto_buf, &a.xcd)) return rc;
    a.state = state; a.u_prev = u_prev; a.pvec = pvec; a.target = target; a.prm = prm; a.w_warm = w_warm;
    a.u0 = u0; a.f = f; a.w_out = w_out; a.status = status; a.iters = iters;
    a.fuse_policy = 0;
    HIPCHK(h, dartmpc_launch_lmpc(&a, stream ? (hipStream_t)stream : h->stream), "kernel launch");
    return DART_MPC_OK;
}

int dart_lmpc_solve_batch(dart_mpc_handle* h, int B, const double* state, const double* u_prev, const double* pvec,
                          const double* target, const double* prm, const double* w_warm, double* u0, double* f,
                          double* w_out, int32_t* status, int32_t* iters, void* stream) {
    if (!h) return DART_MPC_EINVAL;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    if (h->cfg.variant != DART_MPC_LMPC) return fail(h, DART_MPC_EINVAL, "handle is not an LMPC handle");
    if (B < 0 || (B > 0 && (!state || !u_prev || !pvec || !target || !prm || !u0 || !f || !status || !iters)))
        return fail(h, DART_MPC_EINVAL, "null pointer or negative batch");
    if (B > h->cfg.B_max) return fail(h, DART_MPC_EINVAL, "batch larger than B_max");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    const size_t nw = (size_t)dart_lmpc_nw(h->cfg.N);
    HostStage& S = h->st;
    S.begin();
    const double* d_st0 = S.in(state, 8 * B);
    const double* d_up = S.in(u_prev, 2 * B);
    const double* d_pv = S.in(pvec, dartmpc::LM_NPV * B);
    const double* d_tg = S.in(target, 8 * B);
    const double* d_prm = S.in(prm, dartmpc::LM_NPRM * B);
    const double* d_ww = S.in(w_warm, nw * B);
    double* d_u0 = S.out<double>(2 * B);
    double* d_f = S.out<double>(B);
    double* d_wo = w_out ? S.out<double>(nw * B) : nullptr;
    int32_t* d_st = S.out<int32_t>(B);
    int32_t* d_it = S.out<int32_t>(B);
    HIPCHK(h, S.upload(s), "copy inputs");
    int rc = dart_lmpc_solve_batch_dev(h, B, d_st0, d_up, d_pv, d_tg, d_prm, d_ww, d_u0, d_f, d_wo, d_st, d_it, s);
    if (rc) return rc;
    HIPCHK(h, hipStreamSynchronize(s), "hipStreamSynchronize");
    S.take(u0, d_u0, 2 * B); S.take(f, d_f, B); S.take(w_out, d_wo, nw * B);
    S.take(status, d_st, B); S.take(iters, d_it, B);
    return DART_MPC_OK;
}

void dart_lmpc_policy_config_default(dart_lmpc_policy_config* c) {
    if (!c) return;
    c->update_every = 8;
    c->reserved = 0;
    c->max_delta = 0.02;
    c->k_max = 2.0;
    c->min_k = 1e-2;
    c->k_ceiling_margin = std::fmax(1e-3, 0.05 * c->k_max);
    c->action_scale = 1.0;
    c->smooth_alpha = 0.5;
    c->log_std_min = std::log(1e-2);
    c->log_std_max = std::log(2.0);
}

static int policy_args(const dart_lmpc_policy_config* c, int B, const float* w, dartmpc::PolicyArgs& a) {
    if (!c || B < 0 || !w || c->update_every < 1 || !(c->k_max > c->min_k) || !(c->min_k > 0.0)) return DART_MPC_EINVAL;
    a.B = B;
    a.w.W1 = w; a.w.b1 = w + 520 * 64; a.w.W2 = a.w.b1 + 64; a.w.b2 = a.w.W2 + 64 * 64;
    a.w.W3 = a.w.b2 + 64; a.w.b3 = a.w.W3 + 64 * 34; a.w.log_std = a.w.b3 + 34;
    a.update_every = c->update_every;
    a.max_delta = c->max_delta; a.k_max = c->k_max; a.min_k = c->min_k; a.k_ceiling_margin = c->k_ceiling_margin;
    a.action_scale = c->action_scale; a.smooth_alpha = c->smooth_alpha;
    a.log_std_min = c->log_std_min; a.log_std_max = c->log_std_max;
    return DART_MPC_OK;
}

int dart_lmpc_policy_step_dev(const dart_lmpc_policy_config* cfg, int B, const float* weights, const double* state,
                              const double* target, const double* control, const double* current_k, double* obs_mean,
                              double* obs_M2, int32_t* obs_count, float* history, int32_t* timestep, const float* noise,
                              double* model_params, float* action_out, void* stream) {
    dartmpc::PolicyArgs a;
    if (policy_args(cfg, B, weights, a) != DART_MPC_OK) return DART_MPC_EINVAL;
    if (B > 0 && (!state || !target || !control || !current_k || !obs_mean || !obs_M2 || !obs_count || !history ||
                  !timestep || !noise || !model_params)) return DART_MPC_EINVAL;
    if (B == 0) return DART_MPC_OK;
    a.state = state; a.target = target; a.control = control; a.current_k = current_k; a.obs_mean = obs_mean;
    a.obs_M2 = obs_M2; a.obs_count = obs_count; a.history = history; a.timestep = timestep; a.noise = noise;
    a.model_params = model_params; a.action_out = action_out;
    return dartmpc_launch_policy(&a, (hipStream_t)stream) == hipSuccess ? DART_MPC_OK : DART_MPC_EHIP;
}

int dart_lmpc_policy_step(const dart_lmpc_policy_config* cfg, int B, const float* weights, const double* state,
                          const double* target, const double* control, const double* current_k, double* obs_mean,
                          double* obs_M2, int32_t* obs_count, float* history, int32_t* timestep, const float* noise,
                          double* model_params, float* action_out) {
    dartmpc::PolicyArgs a;
    if (policy_args(cfg, B, weights, a) != DART_MPC_OK) return DART_MPC_EINVAL;
    if (B > 0 && (!state || !target || !control || !current_k || !obs_mean || !obs_M2 || !obs_count || !history ||
                  !timestep || !noise || !model_params)) return DART_MPC_EINVAL;
    if (B == 0) return DART_MPC_OK;
    DeviceStage* D = nullptr;
    if (device_stage(&D) != hipSuccess) return DART_MPC_EHIP;
    std::lock_guard<std::mutex> lock(D->mu);
    HostStage& S = D->st;
    const size_t nin = sizeof(float) * ((size_t)DART_LMPC_POLICY_NWEIGHTS + (size_t)B * (34 + 520)) +
                       sizeof(double) * (size_t)B * (8 + 8 + 2 + 34 + 52 + 52 + 34) + sizeof(int32_t) * 2 * B + 16 * 256;
    if (S.reserve(nin, sizeof(float) * 34 * B + 256) != hipSuccess) return DART_MPC_EHIP;
    S.begin();
    const float* d_w = S.in(weights, (size_t)DART_LMPC_POLICY_NWEIGHTS);
    a.w.W1 = d_w; a.w.b1 = d_w + 520 * 64; a.w.W2 = a.w.b1 + 64; a.w.b2 = a.w.W2 + 64 * 64;
    a.w.W3 = a.w.b2 + 64; a.w.b3 = a.w.W3 + 64 * 34; a.w.log_std = a.w.b3 + 34;
    a.state = S.in(state, 8 * (size_t)B); a.target = S.in(target, 8 * (size_t)B);
    a.control = S.in(control, 2 * (size_t)B); a.current_k = S.in(current_k, 34 * (size_t)B);
    a.noise = S.in(noise, 34 * (size_t)B);
    a.obs_mean = S.inout(obs_mean, 52 * (size_t)B); a.obs_M2 = S.inout(obs_M2, 52 * (size_t)B);
    a.model_params = S.inout(model_params, 34 * (size_t)B); a.history = S.inout(history, 520 * (size_t)B);
    a.obs_count = S.inout(obs_count, (size_t)B); a.timestep = S.inout(timestep, (size_t)B);
    a.action_out = S.out<float>(34 * (size_t)B);
    hipError_t e = S.upload(D->stream);
    if (e == hipSuccess) e = dartmpc_launch_policy(&a, D->stream);
    if (e == hipSuccess) e = S.download_inout(D->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(D->stream);
    if (e != hipSuccess) return DART_MPC_EHIP;
    S.finish_inout();
    S.take(action_out, a.action_out, 34 * (size_t)B);
    return DART_MPC_OK;
}


// fused policy step + LMPC solve: one launch (lmpc_ipm.hip prologue = policy_step_wave)
int dart_lmpc_policy_solve_batch_dev(dart_mpc_handle* h, const dart_lmpc_policy_config* pcfg, int B,
                                     const float* weights, const double* state, const double* u_prev,
                                     const double* target, const double* current_k, double* obs_mean, double* obs_M2,
                                     int32_t* obs_count, float* history, int32_t* timestep, const float* noise,
                                     double* model_params, float* action_out, const double* prm, const double* w_warm,
                                     double* u0, double* f, double* w_out, int32_t* status, int32_t* iters,
                                     void* stream) {
    if (!h) return DART_MPC_EINVAL;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    if (h->cfg.variant != DART_MPC_LMPC) return fail(h, DART_MPC_EINVAL, "handle is not an LMPC handle");
    dartmpc::LmpcArgs a;
    if (policy_args(pcfg, B, weights, a.pol) != DART_MPC_OK) return fail(h, DART_MPC_EINVAL, "bad policy config");
    if (B > 0 && (!state || !u_prev || !target || !current_k || !obs_mean || !obs_M2 || !obs_count || !history ||
                  !timestep || !noise || !model_params || !prm || !u0 || !f || !status || !iters))
        return fail(h, DART_MPC_EINVAL, "null pointer");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    a.pol.state = state; a.pol.target = target; a.pol.control = u_prev; a.pol.current_k = current_k;
    a.pol.obs_mean = obs_mean; a.pol.obs_M2 = obs_M2; a.pol.obs_count = obs_count; a.pol.history = history;
    a.pol.timestep = timestep; a.pol.noise = noise; a.pol.model_params = model_params; a.pol.action_out = action_out;
    a.fuse_policy = 1;
    a.B = B; a.N = h->cfg.N; a.Ts = h->cfg.Ts; a.tol = h->cfg.tol; a.max_iter = h->cfg.max_iter;
    a.acc_tol = h->cfg.acceptable_tol; a.acc_iter = h->cfg.acceptable_iter; a.max_soc = h->cfg.max_soc; a.mult_init_max = h->cfg.constr_mult_init_max;
    a.resto = h->cfg.restoration;
    a.max_ticks = (long long)(h->cfg.max_cpu_time * 1e8);     // s_memrealtime: 100 MHz
    if (int rc = stream_state(h, B, stream ? (hipStream_t)stream : h->stream, &a.resto_buf, &a.xcd)) return rc;
    a.state = state; a.u_prev = u_prev; a.pvec = nullptr; a.target = target; a.prm = prm; a.w_warm = w_warm;
    a.u0 = u0; a.f = f; a.w_out = w_out; a.status = status; a.iters = iters;
    HIPCHK(h, dartmpc_launch_lmpc(&a, stream ? (hipStream_t)stream : h->stream), "kernel launch");
    return DART_MPC_OK;
}

int dart_lmpc_policy_solve_batch(dart_mpc_handle* h, const dart_lmpc_policy_config* pcfg, int B, const float* weights,
                                 const double* state, const double* u_prev, const double* target,
                                 const double* current_k, double* obs_mean, double* obs_M2, int32_t* obs_count,
                                 float* history, int32_t* timestep, const float* noise, double* model_params,
                                 float* action_out, const double* prm, const double* w_warm, double* u0, double* f,
                                 double* w_out, int32_t* status, int32_t* iters, void* stream) {
    if (!h) return DART_MPC_EINVAL;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    if (h->cfg.variant != DART_MPC_LMPC) return fail(h, DART_MPC_EINVAL, "handle is not an LMPC handle");
    dartmpc::PolicyArgs chk;
    if (policy_args(pcfg, B, weights, chk) != DART_MPC_OK) return fail(h, DART_MPC_EINVAL, "bad policy config");
    if (B > 0 && (!state || !u_prev || !target || !current_k || !obs_mean || !obs_M2 || !obs_count || !history ||
                  !timestep || !noise || !model_params || !prm || !u0 || !f || !status || !iters))
        return fail(h, DART_MPC_EINVAL, "null pointer");
    if (B > h->cfg.B_max) return fail(h, DART_MPC_EINVAL, "batch larger than B_max");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    const size_t nw = (size_t)dart_lmpc_nw(h->cfg.N), Bz = (size_t)B;
    HostStage& S = h->st;
    const size_t nin = sizeof(float) * ((size_t)DART_LMPC_POLICY_NWEIGHTS + Bz * (34 + 520)) +
                       sizeof(double) * Bz * (8 + 2 + 8 + 34 + dartmpc::LM_NPRM + nw + 52 + 52 + 34) +
                       sizeof(int32_t) * 2 * Bz + 24 * 256;
    const size_t nout = sizeof(double) * Bz * (2 + 1 + nw) + sizeof(int32_t) * 2 * Bz + sizeof(float) * 34 * Bz + 8 * 256;
    HIPCHK(h, S.reserve(nin, nout), "staging buffers");
    S.begin();
    const float* d_w = S.in(weights, (size_t)DART_LMPC_POLICY_NWEIGHTS);
    const double* d_st0 = S.in(state, 8 * Bz);
    const double* d_up = S.in(u_prev, 2 * Bz);
    const double* d_tg = S.in(target, 8 * Bz);
    const double* d_ck = S.in(current_k, 34 * Bz);
    const float* d_nz = S.in(noise, 34 * Bz);
    const double* d_prm = S.in(prm, dartmpc::LM_NPRM * Bz);
    const double* d_ww = S.in(w_warm, nw * Bz);
    double* d_mean = S.inout(obs_mean, 52 * Bz);
    double* d_M2 = S.inout(obs_M2, 52 * Bz);
    double* d_mp = S.inout(model_params, 34 * Bz);
    float* d_hist = S.inout(history, 520 * Bz);
    int32_t* d_cnt = S.inout(obs_count, Bz);
    int32_t* d_ts = S.inout(timestep, Bz);
    double* d_u0 = S.out<double>(2 * Bz);
    double* d_f = S.out<double>(Bz);
    double* d_wo = w_out ? S.out<double>(nw * Bz) : nullptr;
    int32_t* d_stt = S.out<int32_t>(Bz);
    int32_t* d_it = S.out<int32_t>(Bz);
    float* d_act = action_out ? S.out<float>(34 * Bz) : nullptr;
    HIPCHK(h, S.upload(s), "copy inputs");
    int rc = dart_lmpc_policy_solve_batch_dev(h, pcfg, B, d_w, d_st0, d_up, d_tg, d_ck, d_mean, d_M2, d_cnt, d_hist, d_ts,
                                              d_nz, d_mp, d_act, d_prm, d_ww, d_u0, d_f, d_wo, d_stt, d_it, s);
    if (rc) return rc;
    HIPCHK(h, S.download_inout(s), "copy policy state");
    HIPCHK(h, hipStreamSynchronize(s), "hipStreamSynchronize");
    S.finish_inout();
    S.take(u0, d_u0, 2 * Bz); S.take(f, d_f, Bz); S.take(w_out, d_wo, nw * Bz);
    S.take(status, d_stt, Bz); S.take(iters, d_it, Bz); S.take(action_out, d_act, 34 * Bz);
    return DART_MPC_OK;
}

int dart_rls_update_batch_dev(int B, double* theta, double* P, const double* phi, const double* y, double lambda,
                              void* stream) {
    if (B < 0 || (B > 0 && (!theta || !P || !phi || !y)) || !(lambda > 0.0)) return DART_MPC_EINVAL;
    return dartmpc_launch_rls(B, theta, P, phi, y, lambda, (hipStream_t)stream) == hipSuccess ? DART_MPC_OK : DART_MPC_EHIP;
}

int dart_set_device(int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return DART_MPC_ENODEV;
    return hipSetDevice(device) == hipSuccess ? DART_MPC_OK : DART_MPC_EHIP;
}

int dart_rls_update_batch(int B, double* theta, double* P, const double* phi, const double* y, double lambda) {
    if (B < 0 || (B > 0 && (!theta || !P || !phi || !y)) || !(lambda > 0.0)) return DART_MPC_EINVAL;
    if (B == 0) return DART_MPC_OK;
    DeviceStage* D = nullptr;
    if (device_stage(&D) != hipSuccess) return DART_MPC_EHIP;
    std::lock_guard<std::mutex> lock(D->mu);
    HostStage& S = D->st;
    if (S.reserve(sizeof(double) * (size_t)B * (7 + 49 + 7 + 1) + 4 * 256, 256) != hipSuccess) return DART_MPC_EHIP;
    S.begin();
    const double* dphi = S.in(phi, 7 * (size_t)B);
    const double* dy = S.in(y, (size_t)B);
    double* dt = S.inout(theta, 7 * (size_t)B);
    double* dP = S.inout(P, 49 * (size_t)B);
    hipError_t e = S.upload(D->stream);
    if (e == hipSuccess) e = dartmpc_launch_rls(B, dt, dP, dphi, dy, lambda, D->stream);
    if (e == hipSuccess) e = S.download_inout(D->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(D->stream);
    if (e != hipSuccess) return DART_MPC_EHIP;
    S.finish_inout();
    return DART_MPC_OK;
}

int dart_mpc_serve_start(dart_mpc_handle* h, int B_serve, double idle_timeout_s) {
    if (!h) return DART_MPC_EINVAL;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    if (h->cfg.variant != DART_MPC_PMPC) return fail(h, DART_MPC_EINVAL, "handle is not a PMPC handle");
    if (h->cfg.N > 31 || h->cfg.pmpc_path != 0)
        return fail(h, DART_MPC_EINVAL, "the resident server serves IPOPT's path with N <= 31");
    if (B_serve < 1 || B_serve > h->cfg.B_max || B_serve > 65535 || !(idle_timeout_s > 0.0) || idle_timeout_s > 3600.0)
        return fail(h, DART_MPC_EINVAL, "B_serve must be in [1, min(B_max, 65535)], idle timeout in (0, 3600] s");
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    if (int rc = settle_pending(h)) return rc;
    if (int rc = server_stop(h)) return rc;
    HIPCHK(h, ensure_io(h), "I/O area");
    auto& v = h->srv;
    hipError_t e = hipHostMalloc((void**)&v.mbox, 256, hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&v.dmbox, v.mbox, 0);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&v.stream, hipStreamNonBlocking);
    if (e != hipSuccess) { server_release(h); return fail(h, DART_MPC_EHIP, "resident server buffers", e); }
    std::memset(v.mbox, 0, 256);
    v.B = B_serve;
    v.idle_ticks = (unsigned long long)(idle_timeout_s * 1.0e8);      // s_memrealtime: 100 MHz
    v.idle_s = idle_timeout_s;
    v.mbox[0] = h->seq;
    e = server_launch(h, h->seq);
    if (e != hipSuccess) { server_release(h); return fail(h, DART_MPC_EHIP, "resident server launch", e); }
    v.wanted = true;
    return DART_MPC_OK;
}

int dart_mpc_bind(dart_mpc_handle* h, double** x0, double** ref, double** prm, double** w_warm, double** u0, double** f,
                  double** w_out, int32_t** status, int32_t** iters) {
    if (!h) return DART_MPC_EINVAL;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    if (h->cfg.variant != DART_MPC_PMPC) return fail(h, DART_MPC_EINVAL, "handle is not a PMPC handle");
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    HIPCHK(h, ensure_io(h), "I/O area");
    const auto& o = h->io;
    if (x0) *x0 = (double*)o.hin;
    if (ref) *ref = (double*)(o.hin + o.off_ref);
    if (prm) *prm = (double*)(o.hin + o.off_prm);
    if (w_warm) *w_warm = (double*)(o.hin + o.off_ww);
    if (u0) *u0 = (double*)o.hout;
    if (f) *f = (double*)(o.hout + o.off_f);
    if (w_out) *w_out = (double*)(o.hout + o.off_wo);
    if (status) *status = (int32_t*)(o.hout + o.off_st);
    if (iters) *iters = (int32_t*)(o.hout + o.off_it);
    return DART_MPC_OK;
}

int dart_mpc_solve_bound(dart_mpc_handle* h, int B, int flags) {
    if (!h) return DART_MPC_EINVAL;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    if (h->cfg.variant != DART_MPC_PMPC) return fail(h, DART_MPC_EINVAL, "handle is not a PMPC handle");
    if (!h->io.hin) return fail(h, DART_MPC_EINVAL, "dart_mpc_bind first");
    if (B < 0 || B > h->cfg.B_max || (flags & ~3)) return fail(h, DART_MPC_EINVAL, "bad batch or flags");
    if (B == 0) return DART_MPC_OK;
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    if (int rc = settle_pending(h)) return rc;
    const bool ww = flags & DART_MPC_BOUND_W_WARM, wo = flags & DART_MPC_BOUND_W_OUT;
    if (h->srv.wanted && B <= h->srv.B) return served_request(h, B, ww, wo);
    return bound_launch(h, B, ww, wo);
}

int dart_mpc_serve_stop(dart_mpc_handle* h) {
    if (!h) return DART_MPC_EINVAL;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    HIPCHK(h, hipSetDevice(h->device), "hipSetDevice");
    return server_stop(h);
}

int dart_mpc_serve_running(dart_mpc_handle* h) {
    if (!h) return 0;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    if (!h->srv.running) return 0;
    if (hipStreamQuery(h->srv.stream) != hipErrorNotReady) h->srv.running = false;     // idle timeout: drained
    return h->srv.running ? 1 : 0;
}

int dart_mpc_sync(dart_mpc_handle* h) {
    if (!h) return DART_MPC_EINVAL;
    std::unique_lock<std::recursive_mutex> lock_(h->mu);
    if (int rc = settle_pending(h)) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    return DART_MPC_OK;
}

// internal self-test of the wave primitives (not in include/dart_mpc.h): host_out[265]
int dartmpc_selftest(double* host_out) {
    double* d = nullptr;
    if (hipMalloc(&d, 265 * sizeof(double)) != hipSuccess) return DART_MPC_EHIP;
    hipError_t e = dartmpc_wave_selftest(d, nullptr);
    if (e == hipSuccess) e = hipMemcpy(host_out, d, 265 * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? DART_MPC_OK : DART_MPC_EHIP;
}

const char* dart_mpc_last_error(const dart_mpc_handle* h) { return h ? h->err.c_str() : "null handle"; }

void dart_mpc_destroy(dart_mpc_handle* h) {
    if (!h) return;
    (void)server_stop(h);                                     // the resident grid drains first
    if (h->stream) (void)hipStreamSynchronize(h->stream);    // no launch may still use the buffers below
    h->st.release();
    io_release(h);
    if (h->hdone) (void)hipHostFree(h->hdone);
    for (auto& e : h->resto)
        if (e.buf) (void)hipFree(e.buf);       // (synchronises with the area's last use)
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// per-arm impedance QP (ARMCONTROL.solver_worker, PMPC/src/controller/arm.py:266-457)
void dart_arm_config_default(dart_arm_config* c) {
    if (!c) return;
    c->tol = 1e-10;
    c->acceptable_tol = 1e-7;
    c->max_iter = 60;
    c->reserved = 0;
}

int dart_arm_snapshot_len(int n) { return (n >= 1 && n <= DART_ARM_NMAX) ? dartmpc::arm_snap_len(n) : DART_MPC_EINVAL; }
int dart_arm_param_len(int n) { return (n >= 1 && n <= DART_ARM_NMAX) ? dartmpc::arm_prm_len(n) : DART_MPC_EINVAL; }

static int arm_args(const dart_arm_config* c, int B, int n, int prm_stride, dartmpc::ArmArgs& a) {
    if (!c || B < 0 || n < 1 || n > DART_ARM_NMAX) return DART_MPC_EINVAL;
    if (prm_stride != 0 && prm_stride != dartmpc::arm_prm_len(n)) return DART_MPC_EINVAL;
    if (!(c->tol > 0.0) || !(c->acceptable_tol >= c->tol) || c->max_iter < 1 || c->max_iter > 100000) return DART_MPC_EINVAL;
    a = dartmpc::ArmArgs{};
    a.B = B; a.n = n; a.prm_stride = prm_stride; a.max_iter = c->max_iter;
    a.tol = c->tol; a.acc_tol = c->acceptable_tol;
    return DART_MPC_OK;
}

int dart_arm_solve_batch_dev(const dart_arm_config* cfg, int B, int n, const double* snap, const double* prm,
                             int prm_stride, double* qdd, double* tau, double* loss, int32_t* status, int32_t* iters,
                             void* stream) {
    dartmpc::ArmArgs a;
    if (arm_args(cfg, B, n, prm_stride, a) != DART_MPC_OK) return DART_MPC_EINVAL;
    if (B == 0) return DART_MPC_OK;
    if (!snap || !prm || !qdd || !tau || !loss || !status || !iters) return DART_MPC_EINVAL;
    a.snap = snap; a.prm = prm; a.qdd = qdd; a.tau = tau; a.loss = loss; a.status = status; a.iters = iters;
    return dartmpc_launch_arm(&a, (hipStream_t)stream) == hipSuccess ? DART_MPC_OK : DART_MPC_EHIP;
}

int dart_arm_solve_batch(const dart_arm_config* cfg, int B, int n, const double* snap, const double* prm,
                         int prm_stride, double* qdd, double* tau, double* loss, int32_t* status, int32_t* iters) {
    dartmpc::ArmArgs a;
    if (arm_args(cfg, B, n, prm_stride, a) != DART_MPC_OK) return DART_MPC_EINVAL;
    if (B == 0) return DART_MPC_OK;
    if (!snap || !prm || !qdd || !tau || !loss || !status || !iters) return DART_MPC_EINVAL;
    const size_t SL = (size_t)dartmpc::arm_snap_len(n), PL = (size_t)dartmpc::arm_prm_len(n);
    const size_t np = prm_stride ? PL * B : PL;
    DeviceStage* D = nullptr;
    if (device_stage(&D) != hipSuccess) return DART_MPC_EHIP;
    std::lock_guard<std::mutex> lock(D->mu);
    HostStage& S = D->st;
    if (S.reserve(sizeof(double) * (SL * B + np) + 2 * 256,
                  sizeof(double) * (2 * (size_t)n * B + B) + sizeof(int32_t) * 2 * B + 5 * 256) != hipSuccess)
        return DART_MPC_EHIP;
    S.begin();
    a.snap = S.in(snap, SL * B); a.prm = S.in(prm, np);
    a.qdd = S.out<double>((size_t)n * B); a.tau = S.out<double>((size_t)n * B); a.loss = S.out<double>(B);
    a.status = S.out<int32_t>(B); a.iters = S.out<int32_t>(B);
    hipError_t e = S.upload(D->stream);
    if (e == hipSuccess) e = dartmpc_launch_arm(&a, D->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(D->stream);
    if (e != hipSuccess) return DART_MPC_EHIP;
    S.take(qdd, a.qdd, (size_t)n * B); S.take(tau, a.tau, (size_t)n * B); S.take(loss, a.loss, B);
    S.take(status, a.status, B); S.take(iters, a.iters, B);
    return DART_MPC_OK;
}
