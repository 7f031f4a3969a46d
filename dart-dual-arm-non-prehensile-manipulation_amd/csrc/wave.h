// wave.h -- wave64 primitives for gfx950 shared by the solver kernels: DPP lane shifts,
// DPP row reductions, fast reciprocal, cheap log2 and small-angle sin/cos.
#pragma once
#include <stdlib.h>
#include <hip/hip_runtime.h>

namespace dartmpc {

// The lane of the calling thread in its wave64 (= threadIdx.x in the one-wave workgroups of these kernels).
// Code that the restoration tails call uses this instead of threadIdx.x: a non-inlined callee that reads a
// work-item id makes its kernel keep the packed ids live in a VGPR (v31) from entry to the call -- one more live
// register in kernels that sit at the register limit (measured: RMPC C3 -7 %).
__device__ __forceinline__ int lane_id() {
    return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// The launch arguments of the calling kernel for a non-inlined callee (the restoration tails): the kernel passes
// the address of its argument segment (its first argument sits at offset 0) and the callee loads the struct
// from it with scalar loads.  (__builtin_amdgcn_kernarg_segment_ptr is only valid in the kernel itself: in a
// callee it reads 0.)
__device__ __forceinline__ unsigned long long kernarg_addr() {
#if defined(__HIP_DEVICE_COMPILE__)
    return (unsigned long long)__builtin_amdgcn_kernarg_segment_ptr();
#else
    return 0;
#endif
}
// host: the fused restoration (restoration in the solving wave for B <= 32) unless DART_RESTO_FUSE=0 (A/B
// experiments: the round-4 form, a queued restoration kernel behind every launch)
inline bool resto_fuse_enabled() {
    static const bool on = [] {
        const char* e = getenv("DART_RESTO_FUSE");
        return !(e && e[0] == '0');
    }();
    return on;
}
// host, diagnostic: DART_FORCE_WG2=1 runs RMPC and LMPC on their two-wave builds at every N (A/B of the two-wave
// machinery against the one-wave kernels on the same instances; tools/wg2_ab.py)
inline bool force_wg2() {
    static const bool on = [] {
        const char* e = getenv("DART_FORCE_WG2");
        return e && e[0] == '1';
    }();
    return on;
}
template <class T>
__device__ __forceinline__ T kernarg_load(unsigned long long addr) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const T __attribute__((address_space(4))) KernT;
    return *(KernT*)addr;
#else
    (void)addr;
    return T{};
#endif
}

constexpr int kWave = 64;

// Waves per instance.  1: the kernels as written (one wave64 per instance, lane k and k + 32 own node k, N <= 31).
// 2: the DART_WG=2 builds of the RMPC and LMPC kernels for N = 32..63 -- a workgroup of two waves, wave w owns
// nodes 32 w .. 32 w + 31 with the one-wave lane roles.  There every wave reduction below and the node shifts
// from_prev / from_next combine the two waves through LDS (two barriers each), and the node-coupled sweeps of
// ocp_wave.h run redundantly in both waves on the shared LDS data (equal values written twice), so the solver
// code above these primitives is the one-wave code.
#ifndef DART_WG
#define DART_WG 1
#endif
constexpr int kWaves = DART_WG;
static_assert(kWaves == 1 || kWaves == 2, "one or two waves per instance");

__device__ __forceinline__ int wave_idx() {
#if DART_WG == 2
    return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
#else
    return 0;
#endif
}
// the first node of the calling wave
__device__ __forceinline__ int node_base() { return 32 * wave_idx(); }

#if DART_WG == 2
__shared__ double g_wg_x[2][8];
// wave-uniform values of both waves, o[w][i] = v[i] of wave w; every wave then combines them in wave order (the
// same result in both).  The second barrier keeps the next exchange from overwriting a slot still to be read.
template <int NV>
__device__ __forceinline__ void wg_both(const double (&v)[NV], double (&o)[2][NV]) {
    static_assert(NV <= 8, "eight slots");
    const int w = wave_idx();
    if (lane_id() == 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) g_wg_x[w][i] = v[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) { o[0][i] = g_wg_x[0][i]; o[1][i] = g_wg_x[1][i]; }
    __syncthreads();
}
#endif

// ---------------------------------------------------------------------------
// wave primitives (every call site is at wave-uniform control flow: EXEC full)
// ---------------------------------------------------------------------------
// DPP move with bound_ctrl: lanes whose source is out of range get 0, rows masked off by ROWMASK
// are left undefined (no initialising copy of the destination is needed either way)
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ double dpp(double x) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
    const int lo = (int)(unsigned)(b & 0xffffffffu), hi = (int)(unsigned)(b >> 32);
    const int rlo = __builtin_amdgcn_mov_dpp(lo, CTRL, ROWMASK, 0xf, true);
    const int rhi = __builtin_amdgcn_mov_dpp(hi, CTRL, ROWMASK, 0xf, true);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)rhi << 32) | (unsigned)rlo);
}
__device__ __forceinline__ double readlane(double x, int l) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)(b & 0xffffffffu), l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// value of lane 16 (lane / 16) + I in every lane of each 16-lane row: one v_mov_b64_dpp
// row_newbcast (the 64-bit DPP control of gfx950), no scalar round trip and no LDS crossbar
template <int I>
__device__ __forceinline__ double row_bcast(double x) {
    return __builtin_amdgcn_update_dpp(0.0, x, 0x150 + I, 0xf, 0xf, false);
}
// the same with the destination's dead previous value as the DPP "old" operand: every lane reads a
// valid source under row_newbcast, so old never shows, and tying it to the destination spares the
// initialising move that an explicit old value costs
template <int I>
__device__ __forceinline__ double row_bcast_over(double x, double dead) {
    return __builtin_amdgcn_update_dpp(dead, x, 0x150 + I, 0xf, 0xf, false);
}
__device__ __forceinline__ double row_bcast_over(double x, int i, double dead) {
    switch (i) {       // i (< 8) is a compile-time constant at every (unrolled) call site
        case 0: return row_bcast_over<0>(x, dead);
        case 1: return row_bcast_over<1>(x, dead);
        case 2: return row_bcast_over<2>(x, dead);
        case 3: return row_bcast_over<3>(x, dead);
        case 4: return row_bcast_over<4>(x, dead);
        case 5: return row_bcast_over<5>(x, dead);
        case 6: return row_bcast_over<6>(x, dead);
        default: return row_bcast_over<7>(x, dead);
    }
}
__device__ __forceinline__ double row_bcast(double x, int i) {
    switch (i) {       // i (< 8) is a compile-time constant at every (unrolled) call site
        case 0: return row_bcast<0>(x);
        case 1: return row_bcast<1>(x);
        case 2: return row_bcast<2>(x);
        case 3: return row_bcast<3>(x);
        case 4: return row_bcast<4>(x);
        case 5: return row_bcast<5>(x);
        case 6: return row_bcast<6>(x);
        default: return row_bcast<7>(x);
    }
}
// value of lane 32 (lane / 32) + I in every lane of each 32-lane half: ds_swizzle bitmask mode
// (and_mask 0, or_mask I) -- a crossbar move through the LDS unit without a memory access
template <int I>
__device__ __forceinline__ double half_bcast_c(double x) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
    const int lo = __builtin_amdgcn_ds_swizzle((int)(unsigned)(b & 0xffffffffu), I << 5);
    const int hi = __builtin_amdgcn_ds_swizzle((int)(unsigned)(b >> 32), I << 5);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double half_bcast(double x, int i) {
    switch (i) {       // i (< 16) is a compile-time constant at every (unrolled) call site
        case 0: return half_bcast_c<0>(x);
        case 1: return half_bcast_c<1>(x);
        case 2: return half_bcast_c<2>(x);
        case 3: return half_bcast_c<3>(x);
        case 4: return half_bcast_c<4>(x);
        case 5: return half_bcast_c<5>(x);
        case 6: return half_bcast_c<6>(x);
        case 7: return half_bcast_c<7>(x);
        case 8: return half_bcast_c<8>(x);
        case 9: return half_bcast_c<9>(x);
        case 10: return half_bcast_c<10>(x);
        case 11: return half_bcast_c<11>(x);
        case 12: return half_bcast_c<12>(x);
        case 13: return half_bcast_c<13>(x);
        case 14: return half_bcast_c<14>(x);
        default: return half_bcast_c<15>(x);
    }
}
// x[i] + x[i + 32] in lane i and lane i + 32 (the two 32-lane halves summed pairwise): two
// v_permlane32_swap_b32 (gfx950 VALU, no LDS crossbar) exchange lanes 32-63 of one copy with lanes
// 0-31 of the other, after which the two copies hold the low and the high half in every lane; the
// sum needs no select and is the same value (low + high) in both lanes of a pair
__device__ __forceinline__ double half_pair_sum(double x) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
    const unsigned lo = (unsigned)(b & 0xffffffffu), hi = (unsigned)(b >> 32);
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const double a = __builtin_bit_cast(double, ((unsigned long long)rh[0] << 32) | rl[0]);
    const double c = __builtin_bit_cast(double, ((unsigned long long)rh[1] << 32) | rl[1]);
    return a + c;
}
// both values of a lane pair (l mod 32, l mod 32 + 32) in every lane: lo from lanes 0-31, hi from lanes
// 32-63, by the same v_permlane32_swap_b32 pair as half_pair_sum (EXEC must be full)
__device__ __forceinline__ void half_pair(double x, double& lo, double& hi) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
    const unsigned l32 = (unsigned)(b & 0xffffffffu), h32 = (unsigned)(b >> 32);
    const auto rl = __builtin_amdgcn_permlane32_swap(l32, l32, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(h32, h32, false, false);
    lo = __builtin_bit_cast(double, ((unsigned long long)rh[0] << 32) | rl[0]);
    hi = __builtin_bit_cast(double, ((unsigned long long)rh[1] << 32) | rl[1]);
}
constexpr int kWaveShl1 = 0x130;   // lane k <- lane k+1 (lane 63 <- 0)
constexpr int kWaveShr1 = 0x138;   // lane k <- lane k-1 (lane 0 <- 0)
#if DART_WG == 1
__device__ __forceinline__ double from_next(double x) { return dpp<kWaveShl1>(x); }
__device__ __forceinline__ double from_prev(double x) { return dpp<kWaveShr1>(x); }
#else
// two waves: lanes 0 / 32 of wave 1 take lanes 31 / 63 of wave 0 (node 31 of either lane half), and back
__device__ __forceinline__ double from_next(double x) {
    double v = dpp<kWaveShl1>(x);
    const int l = lane_id(), w = wave_idx();
    if (l == 0 || l == 32) g_wg_x[w][l >> 5] = x;
    __syncthreads();
    const double b0 = g_wg_x[1][0], b1 = g_wg_x[1][1];
    __syncthreads();
    if (w == 0 && l == 31) v = b0;
    if (w == 0 && l == 63) v = b1;
    return v;
}
__device__ __forceinline__ double from_prev(double x) {
    double v = dpp<kWaveShr1>(x);
    const int l = lane_id(), w = wave_idx();
    if (l == 31 || l == 63) g_wg_x[w][l >> 5] = x;
    __syncthreads();
    const double b0 = g_wg_x[0][0], b1 = g_wg_x[0][1];
    __syncthreads();
    if (w == 1 && l == 0) v = b0;
    if (w == 1 && l == 32) v = b1;
    return v;
}
#endif

// NV node shifts at once: one wave, the DPP shifts of from_next / from_prev; two waves, one LDS exchange for all
// NV values (two barriers) instead of one per value
#if DART_WG == 2
__shared__ double g_wg_s[2][2][8];        // [wave][lane half][value]
#endif
template <int NV>
__device__ __forceinline__ void from_next_n(const double (&x)[NV], double (&o)[NV]) {
#if DART_WG == 1
#pragma unroll
    for (int i = 0; i < NV; ++i) o[i] = from_next(x[i]);
#else
    static_assert(NV <= 8, "eight slots");
    const int l = lane_id(), w = wave_idx();
#pragma unroll
    for (int i = 0; i < NV; ++i) o[i] = dpp<kWaveShl1>(x[i]);
    if (l == 0 || l == 32) {
#pragma unroll
        for (int i = 0; i < NV; ++i) g_wg_s[w][l >> 5][i] = x[i];
    }
    __syncthreads();
    if (w == 0 && (l == 31 || l == 63)) {
#pragma unroll
        for (int i = 0; i < NV; ++i) o[i] = g_wg_s[1][l >> 5][i];
    }
    __syncthreads();
#endif
}
template <int NV>
__device__ __forceinline__ void from_prev_n(const double (&x)[NV], double (&o)[NV]) {
#if DART_WG == 1
#pragma unroll
    for (int i = 0; i < NV; ++i) o[i] = from_prev(x[i]);
#else
    static_assert(NV <= 8, "eight slots");
    const int l = lane_id(), w = wave_idx();
#pragma unroll
    for (int i = 0; i < NV; ++i) o[i] = dpp<kWaveShr1>(x[i]);
    if (l == 31 || l == 63) {
#pragma unroll
        for (int i = 0; i < NV; ++i) g_wg_s[w][l >> 5][i] = x[i];
    }
    __syncthreads();
    if (w == 1 && (l == 0 || l == 32)) {
#pragma unroll
        for (int i = 0; i < NV; ++i) o[i] = g_wg_s[0][l >> 5][i];
    }
    __syncthreads();
#endif
}

struct OpSum { __device__ double operator()(double a, double b) const { return a + b; } };
struct OpMax { __device__ double operator()(double a, double b) const { return fmax(a, b); } };
struct OpMin { __device__ double operator()(double a, double b) const { return fmin(a, b); } };

// row reduction by quad_perm + row_ror (every lane of a row holds the row total), then the rows
// chained by row_bcast:15 (rows 1, 3 take lane 15 / 47) and row_bcast:31 (rows 2, 3 take lane 31):
// lane 63 holds the wave total, read once (uniform result)
// (BCAST = false: the four row totals by readlane instead -- fewer VGPRs live across the reduction,
// for kernels at the register limit)
template <class Op, bool BCAST = true>
__device__ __forceinline__ double wreduce(double x, Op op) {
    x = op(x, dpp<0xB1>(x));     // quad_perm [1,0,3,2]
    x = op(x, dpp<0x4E>(x));     // quad_perm [2,3,0,1]
    x = op(x, dpp<0x124>(x));    // row_ror:4
    x = op(x, dpp<0x128>(x));    // row_ror:8
    double r;
    if constexpr (!BCAST) {
        r = op(op(readlane(x, 0), readlane(x, 16)), op(readlane(x, 32), readlane(x, 48)));
    } else {
        x = op(x, dpp<0x142, 0xa>(x));   // row_bcast:15
        x = op(x, dpp<0x143, 0xc>(x));   // row_bcast:31
        r = readlane(x, 63);
    }
#if DART_WG == 2
    { const double v[1] = {r}; double o[2][1]; wg_both(v, o); r = op(o[0][0], o[1][0]); }
#endif
    return r;
}
// f32 variant for error measures, scalings and step-length minima (half the DPP traffic):
// their consumers only compare against tolerances or fractions-to-the-boundary with >= 1 % slack
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ float dppf(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, ROWMASK, 0xf, true));
}
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ unsigned dppu(unsigned x) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)x, CTRL, ROWMASK, 0xf, true);
}
__device__ __forceinline__ float readlanef(float x, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}
template <class Op>
__device__ __forceinline__ float wreducef(float x, Op op) {
    x = op(x, dppf<0xB1>(x));
    x = op(x, dppf<0x4E>(x));
    x = op(x, dppf<0x124>(x));
    x = op(x, dppf<0x128>(x));
    x = op(x, dppf<0x142, 0xa>(x));
    x = op(x, dppf<0x143, 0xc>(x));
    float r = readlanef(x, 63);
#if DART_WG == 2
    { const double v[1] = {(double)r}; double o[2][1]; wg_both(v, o); r = op((float)o[0][0], (float)o[1][0]); }
#endif
    return r;
}
struct OpSumF { __device__ float operator()(float a, float b) const { return a + b; } };
struct OpMaxF { __device__ float operator()(float a, float b) const { return fmaxf(a, b); } };
struct OpMinF { __device__ float operator()(float a, float b) const { return fminf(a, b); } };
__device__ __forceinline__ float wsumf(float x) { return wreducef(x, OpSumF()); }
// max / min over the wave of NON-NEGATIVE floats (+0, positive, inf; a NaN propagates as the
// largest): on such values the IEEE order is the unsigned order of the bit patterns, so the steps
// run on v_max_u32 / v_min_u32, without the NaN-quieting canonicalize fmaxf needs on DPP results
struct OpMaxU { __device__ unsigned operator()(unsigned a, unsigned b) const { return a > b ? a : b; } };
struct OpMinU { __device__ unsigned operator()(unsigned a, unsigned b) const { return a < b ? a : b; } };
template <class Op>
__device__ __forceinline__ float wreduce_nn(float xf, Op op) {
    unsigned x = __builtin_bit_cast(unsigned, xf);
    x = op(x, dppu<0xB1>(x));
    x = op(x, dppu<0x4E>(x));
    x = op(x, dppu<0x124>(x));
    x = op(x, dppu<0x128>(x));
    x = op(x, dppu<0x142, 0xa>(x));
    x = op(x, dppu<0x143, 0xc>(x));
    unsigned r = (unsigned)__builtin_amdgcn_readlane((int)x, 63);
#if DART_WG == 2
    { const double v[1] = {(double)r}; double o[2][1]; wg_both(v, o); r = op((unsigned)o[0][0], (unsigned)o[1][0]); }
#endif
    return __builtin_bit_cast(float, r);
}
__device__ __forceinline__ float wmaxf(float x) { return wreduce_nn(x, OpMaxU()); }
__device__ __forceinline__ float wminf(float x) { return wreduce_nn(x, OpMinU()); }

// Several independent reductions advanced level by level in lock step: the chains interleave, so
// no DPP read waits on the VALU result just before it and each chain's latency hides behind the
// others'.  Levels: quad_perm [1,0,3,2], [2,3,0,1], row_ror 4, 8, row_bcast 15 (rows 1, 3),
// row_bcast 31 (rows 2, 3); the total is read from lane 63.
template <int CTRL, int RM>
__device__ __forceinline__ void lvl_sum(double& x) { x += dpp<CTRL, RM>(x); }
template <int CTRL, int RM>
__device__ __forceinline__ void lvl_sumf(float& x) { x += dppf<CTRL, RM>(x); }
template <int CTRL, int RM>
__device__ __forceinline__ void lvl_maxu(unsigned& x) { const unsigned y = dppu<CTRL, RM>(x); x = x > y ? x : y; }
template <int CTRL, int RM>
__device__ __forceinline__ void lvl_minu(unsigned& x) { const unsigned y = dppu<CTRL, RM>(x); x = x < y ? x : y; }
#define DART_LEVELS(F) F(0xB1, 0xf) F(0x4E, 0xf) F(0x124, 0xf) F(0x128, 0xf) F(0x142, 0xa) F(0x143, 0xc)

// two f64 sums
__device__ __forceinline__ void wsum2(double& a, double& b) {
#define DART_L(C, R) lvl_sum<C, R>(a); lvl_sum<C, R>(b);
    DART_LEVELS(DART_L)
#undef DART_L
    a = readlane(a, 63); b = readlane(b, 63);
#if DART_WG == 2
    { const double v[2] = {a, b}; double o[2][2]; wg_both(v, o); a = o[0][0] + o[1][0]; b = o[0][1] + o[1][1]; }
#endif
}
// two f64 sums and one f32 maximum of non-negative values (wreduce_nn) together: two waves, one exchange
__device__ __forceinline__ void wsum2_maxf(double& a, double& b, float& m) {
#if DART_WG == 1
    // one wave: the three chains in lock step (each takes its own wsum / wmaxf steps: the same bits)
    unsigned x = __builtin_bit_cast(unsigned, m);
#define DART_L(C, R) lvl_sum<C, R>(a); lvl_sum<C, R>(b); lvl_maxu<C, R>(x);
    DART_LEVELS(DART_L)
#undef DART_L
    a = readlane(a, 63); b = readlane(b, 63);
    m = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)x, 63));
#else
    unsigned x = __builtin_bit_cast(unsigned, m);
#define DART_L(C, R) lvl_sum<C, R>(a); lvl_sum<C, R>(b); lvl_maxu<C, R>(x);
    DART_LEVELS(DART_L)
#undef DART_L
    a = readlane(a, 63); b = readlane(b, 63);
    x = (unsigned)__builtin_amdgcn_readlane((int)x, 63);
    const double v[3] = {a, b, (double)x};
    double o[2][3];
    wg_both(v, o);
    a = o[0][0] + o[1][0]; b = o[0][1] + o[1][1];
    m = __builtin_bit_cast(float, (unsigned)fmax(o[0][2], o[1][2]));
#endif
}
// wsum2_maxf with two f32 minima of non-negative values (wmin2f) in the same lock step (one wave); two waves: the
// minima first, then wsum2_maxf's exchange
__device__ __forceinline__ void wmin2f(float& a, float& b);
__device__ __forceinline__ void wsum2_maxf_min2f(double& a, double& b, float& m, float& n0, float& n1) {
#if DART_WG == 1
    unsigned x = __builtin_bit_cast(unsigned, m);
    unsigned y0 = __builtin_bit_cast(unsigned, n0), y1 = __builtin_bit_cast(unsigned, n1);
#define DART_L(C, R) lvl_sum<C, R>(a); lvl_sum<C, R>(b); lvl_maxu<C, R>(x); lvl_minu<C, R>(y0); lvl_minu<C, R>(y1);
    DART_LEVELS(DART_L)
#undef DART_L
    a = readlane(a, 63); b = readlane(b, 63);
    m = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)x, 63));
    n0 = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)y0, 63));
    n1 = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)y1, 63));
#else
    wmin2f(n0, n1);
    wsum2_maxf(a, b, m);
#endif
}
// two f32 minima of non-negative values (see wreduce_nn)
__device__ __forceinline__ void wmin2f(float& a, float& b) {
    unsigned x = __builtin_bit_cast(unsigned, a), y = __builtin_bit_cast(unsigned, b);
#define DART_L(C, R) lvl_minu<C, R>(x); lvl_minu<C, R>(y);
    DART_LEVELS(DART_L)
#undef DART_L
#if DART_WG == 2
    x = (unsigned)__builtin_amdgcn_readlane((int)x, 63); y = (unsigned)__builtin_amdgcn_readlane((int)y, 63);
    {
        const double v[2] = {(double)x, (double)y};
        double o[2][2];
        wg_both(v, o);
        x = (unsigned)fmin(o[0][0], o[1][0]); y = (unsigned)fmin(o[0][1], o[1][1]);
    }
    a = __builtin_bit_cast(float, x); b = __builtin_bit_cast(float, y);
#else
    a = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)x, 63));
    b = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)y, 63));
#endif
}
#if DART_WG == 2
// the two waves' error measures combined (maxima / minimum of non-negative floats by their bit patterns)
__device__ __forceinline__ void wg_errors(float& mx0, float& mx1, float& mx2, float* mx3, float& mn, float& s0, float& s1) {
    auto u = [](float f) { return (double)__builtin_bit_cast(unsigned, f); };
    auto f = [](double d) { return __builtin_bit_cast(float, (unsigned)d); };
    const double v[7] = {u(mx0), u(mx1), u(mx2), mx3 ? u(*mx3) : 0.0, u(mn), (double)s0, (double)s1};
    double o[2][7];
    wg_both(v, o);
    mx0 = f(fmax(o[0][0], o[1][0])); mx1 = f(fmax(o[0][1], o[1][1])); mx2 = f(fmax(o[0][2], o[1][2]));
    if (mx3) *mx3 = f(fmax(o[0][3], o[1][3]));
    mn = f(fmin(o[0][4], o[1][4]));
    s0 = (float)o[0][5] + (float)o[1][5]; s1 = (float)o[0][6] + (float)o[1][6];
}
#endif
// the error-measure reductions of an IPM iteration: four maxima and one minimum of non-negative
// values, two f32 sums
__device__ __forceinline__ void wred_errors4(float& mx0, float& mx1, float& mx2, float& mx3, float& mn, float& s0,
                                             float& s1) {
    unsigned a = __builtin_bit_cast(unsigned, mx0), b = __builtin_bit_cast(unsigned, mx1);
    unsigned c = __builtin_bit_cast(unsigned, mx2), e = __builtin_bit_cast(unsigned, mx3);
    unsigned d = __builtin_bit_cast(unsigned, mn);
#define DART_L(C, R) lvl_maxu<C, R>(a); lvl_maxu<C, R>(b); lvl_maxu<C, R>(c); lvl_maxu<C, R>(e); \
    lvl_minu<C, R>(d); lvl_sumf<C, R>(s0); lvl_sumf<C, R>(s1);
    DART_LEVELS(DART_L)
#undef DART_L
    mx0 = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)a, 63));
    mx1 = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)b, 63));
    mx2 = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)c, 63));
    mx3 = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)e, 63));
    mn = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)d, 63));
    s0 = readlanef(s0, 63); s1 = readlanef(s1, 63);
#if DART_WG == 2
    wg_errors(mx0, mx1, mx2, &mx3, mn, s0, s1);
#endif
}
// the error-measure reductions of an IPM iteration: three maxima and one minimum of non-negative
// values, two f32 sums
__device__ __forceinline__ void wred_errors(float& mx0, float& mx1, float& mx2, float& mn, float& s0, float& s1) {
    unsigned a = __builtin_bit_cast(unsigned, mx0), b = __builtin_bit_cast(unsigned, mx1);
    unsigned c = __builtin_bit_cast(unsigned, mx2), d = __builtin_bit_cast(unsigned, mn);
#define DART_L(C, R) lvl_maxu<C, R>(a); lvl_maxu<C, R>(b); lvl_maxu<C, R>(c); lvl_minu<C, R>(d); \
    lvl_sumf<C, R>(s0); lvl_sumf<C, R>(s1);
    DART_LEVELS(DART_L)
#undef DART_L
    mx0 = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)a, 63));
    mx1 = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)b, 63));
    mx2 = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)c, 63));
    mn = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)d, 63));
    s0 = readlanef(s0, 63); s1 = readlanef(s1, 63);
#if DART_WG == 2
    wg_errors(mx0, mx1, mx2, nullptr, mn, s0, s1);
#endif
}

__device__ __forceinline__ double wsum(double x) { return wreduce(x, OpSum()); }
__device__ __forceinline__ double wmax(double x) { return wreduce(x, OpMax()); }
__device__ __forceinline__ double wmin(double x) { return wreduce(x, OpMin()); }
// f64 reductions advanced level by level together (the chains interleave): each value takes exactly the steps of
// its own wsum / wmax / wmin, so the results are the same bits.  The two-wave builds take them one by one.
template <int CTRL, int RM>
__device__ __forceinline__ void lvl_maxd(double& x) { x = fmax(x, dpp<CTRL, RM>(x)); }
template <int CTRL, int RM>
__device__ __forceinline__ void lvl_mind(double& x) { x = fmin(x, dpp<CTRL, RM>(x)); }
// two f64 minima in lock step (the same bits as two wmin)
__device__ __forceinline__ void wmin2d(double& a, double& b) {
#if DART_WG == 1
#define DART_L(C, R) lvl_mind<C, R>(a); lvl_mind<C, R>(b);
    DART_LEVELS(DART_L)
#undef DART_L
    a = readlane(a, 63); b = readlane(b, 63);
#else
    a = wmin(a); b = wmin(b);
#endif
}
__device__ __forceinline__ void wsum3(double& a, double& b, double& c) {
#if DART_WG == 1
#define DART_L(C, R) lvl_sum<C, R>(a); lvl_sum<C, R>(b); lvl_sum<C, R>(c);
    DART_LEVELS(DART_L)
#undef DART_L
    a = readlane(a, 63); b = readlane(b, 63); c = readlane(c, 63);
#else
    a = wsum(a); b = wsum(b); c = wsum(c);
#endif
}
// three maxima, one minimum, two sums (IPOPT's optimality error and its scalings)
__device__ __forceinline__ void wred_errors_f64(double& mx0, double& mx1, double& mx2, double& mn, double& s0, double& s1) {
#if DART_WG == 1
#define DART_L(C, R) lvl_maxd<C, R>(mx0); lvl_maxd<C, R>(mx1); lvl_maxd<C, R>(mx2); lvl_mind<C, R>(mn); \
    lvl_sum<C, R>(s0); lvl_sum<C, R>(s1);
    DART_LEVELS(DART_L)
#undef DART_L
    mx0 = readlane(mx0, 63); mx1 = readlane(mx1, 63); mx2 = readlane(mx2, 63); mn = readlane(mn, 63);
    s0 = readlane(s0, 63); s1 = readlane(s1, 63);
#else
    mx0 = wmax(mx0); mx1 = wmax(mx1); mx2 = wmax(mx2); mn = wmin(mn); s0 = wsum(s0); s1 = wsum(s1);
#endif
}
__device__ __forceinline__ double wsum_rl(double x) { return wreduce<OpSum, false>(x, OpSum()); }
// two wsum_rl (and a wmaxf) in lock step, one wave: each value takes its own reduction's steps (the same bits)
__device__ __forceinline__ void wsum2_rl(double& a, double& b) {
#if DART_WG == 1
#define DART_L(C, R) lvl_sum<C, R>(a); lvl_sum<C, R>(b);
    DART_L(0xB1, 0xf) DART_L(0x4E, 0xf) DART_L(0x124, 0xf) DART_L(0x128, 0xf)
#undef DART_L
    a = (readlane(a, 0) + readlane(a, 16)) + (readlane(a, 32) + readlane(a, 48));
    b = (readlane(b, 0) + readlane(b, 16)) + (readlane(b, 32) + readlane(b, 48));
#else
    a = wsum_rl(a); b = wsum_rl(b);
#endif
}
// wmax x3, wmin and wsum_rl x2 in lock step (RMPC's restoration errors): the same bits as the six calls
__device__ __forceinline__ void wred_errors_f64_rl(double& mx0, double& mx1, double& mx2, double& mn, double& s0, double& s1) {
#if DART_WG == 1
#define DART_L(C, R) lvl_maxd<C, R>(mx0); lvl_maxd<C, R>(mx1); lvl_maxd<C, R>(mx2); lvl_mind<C, R>(mn); \
    lvl_sum<C, R>(s0); lvl_sum<C, R>(s1);
    DART_L(0xB1, 0xf) DART_L(0x4E, 0xf) DART_L(0x124, 0xf) DART_L(0x128, 0xf)
#undef DART_L
#define DART_L(C, R) lvl_maxd<C, R>(mx0); lvl_maxd<C, R>(mx1); lvl_maxd<C, R>(mx2); lvl_mind<C, R>(mn);
    DART_L(0x142, 0xa) DART_L(0x143, 0xc)
#undef DART_L
    mx0 = readlane(mx0, 63); mx1 = readlane(mx1, 63); mx2 = readlane(mx2, 63); mn = readlane(mn, 63);
    s0 = (readlane(s0, 0) + readlane(s0, 16)) + (readlane(s0, 32) + readlane(s0, 48));
    s1 = (readlane(s1, 0) + readlane(s1, 16)) + (readlane(s1, 32) + readlane(s1, 48));
#else
    mx0 = wmax(mx0); mx1 = wmax(mx1); mx2 = wmax(mx2); mn = wmin(mn); s0 = wsum_rl(s0); s1 = wsum_rl(s1);
#endif
}
__device__ __forceinline__ void wsum2_rl_maxf(double& a, double& b, float& m) {
#if DART_WG == 1
    unsigned x = __builtin_bit_cast(unsigned, m);
#define DART_L(C, R) lvl_sum<C, R>(a); lvl_sum<C, R>(b); lvl_maxu<C, R>(x);
    DART_L(0xB1, 0xf) DART_L(0x4E, 0xf) DART_L(0x124, 0xf) DART_L(0x128, 0xf)
#undef DART_L
    lvl_maxu<0x142, 0xa>(x); lvl_maxu<0x143, 0xc>(x);
    a = (readlane(a, 0) + readlane(a, 16)) + (readlane(a, 32) + readlane(a, 48));
    b = (readlane(b, 0) + readlane(b, 16)) + (readlane(b, 32) + readlane(b, 48));
    m = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_readlane((int)x, 63));
#else
    a = wsum_rl(a); b = wsum_rl(b); m = wmaxf(m);
#endif
}
__device__ __forceinline__ bool wany(bool p) {
    bool r = __ballot(p) != 0ull;
#if DART_WG == 2
    { const double v[1] = {r ? 1.0 : 0.0}; double o[2][1]; wg_both(v, o); r = o[0][0] + o[1][0] > 0.0; }
#endif
    return r;
}

// any over the wave of a predicate on state that both waves of a two-wave instance hold alike (the filter
// entries, one per lane, set from wave-uniform values): the wave's own ballot decides, no exchange
__device__ __forceinline__ bool wany_rep(bool p) { return __ballot(p) != 0ull; }

// reciprocal: v_rcp_f64 (measured max relative error 2e-8 on gfx950, tests/test_gpu_pmpc.py
// selftest) + one Newton step -> ~4e-16 relative; operands are well scaled, no denormals
__device__ __forceinline__ double frcp(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    return fma(r, fma(-x, r, 1.0), r);
}

// log2 of a positive double to ~1e-7 relative: exponent + f32 log2 of the mantissa.  Used only in
// the filter's switching condition / minimum step heuristics, never in a quantity that is solved for.
__device__ __forceinline__ float lg2(double x) {
    const int e = __builtin_amdgcn_frexp_exp(x);
    const float m = (float)__builtin_amdgcn_frexp_mant(x);
    return (float)e + __builtin_amdgcn_logf(m);
}

// sin/cos for |x| <= 1.0 (bound-relaxed tilt range) by Taylor series to x^19 / x^20:
// truncation < 2e-20, i.e. below fp64 rounding.  Wider boxes fall back to ocml sincos.
__device__ __forceinline__ void sincos_small(double x, double& s, double& c) {
    const double y = x * x;
    double ps = -1.0 / 121645100408832000.0;                 // -1/19!
    ps = fma(ps, y, 1.0 / 355687428096000.0);                // 1/17!
    ps = fma(ps, y, -1.0 / 1307674368000.0);                 // -1/15!
    ps = fma(ps, y, 1.0 / 6227020800.0);                     // 1/13!
    ps = fma(ps, y, -1.0 / 39916800.0);                      // -1/11!
    ps = fma(ps, y, 1.0 / 362880.0);                         // 1/9!
    ps = fma(ps, y, -1.0 / 5040.0);                          // -1/7!
    ps = fma(ps, y, 1.0 / 120.0);                            // 1/5!
    ps = fma(ps, y, -1.0 / 6.0);                             // -1/3!
    s = fma(x * y, ps, x);
    double pc = 1.0 / 2432902008176640000.0;                 // 1/20!
    pc = fma(pc, y, -1.0 / 6402373705728000.0);              // -1/18!
    pc = fma(pc, y, 1.0 / 20922789888000.0);                 // 1/16!
    pc = fma(pc, y, -1.0 / 87178291200.0);                   // -1/14!
    pc = fma(pc, y, 1.0 / 479001600.0);                      // 1/12!
    pc = fma(pc, y, -1.0 / 3628800.0);                       // -1/10!
    pc = fma(pc, y, 1.0 / 40320.0);                          // 1/8!
    pc = fma(pc, y, -1.0 / 720.0);                           // -1/6!
    pc = fma(pc, y, 1.0 / 24.0);                             // 1/4!
    pc = fma(pc, y, -0.5);                                   // -1/2!
    c = fma(y, pc, 1.0);
}
__device__ __forceinline__ double cos_small(double x) {       // the cosine half of sincos_small
    const double y = x * x;
    double pc = 1.0 / 2432902008176640000.0;
    pc = fma(pc, y, -1.0 / 6402373705728000.0);
    pc = fma(pc, y, 1.0 / 20922789888000.0);
    pc = fma(pc, y, -1.0 / 87178291200.0);
    pc = fma(pc, y, 1.0 / 479001600.0);
    pc = fma(pc, y, -1.0 / 3628800.0);
    pc = fma(pc, y, 1.0 / 40320.0);
    pc = fma(pc, y, -1.0 / 720.0);
    pc = fma(pc, y, 1.0 / 24.0);
    pc = fma(pc, y, -0.5);
    return fma(y, pc, 1.0);
}
// sin/cos for |x| <= 1.0 (bound-relaxed tilt range): the Taylor series to x^23 / x^22, economised
// on [-1, 1] by Chebyshev polynomials to degree 15 (sin) / 16 (cos): truncation <= 4.3e-20 /
// 2.1e-21, <= 1.05 ulp in double with fma Horner -- the accuracy of the degree-19 / 20 Taylor
// polynomials above with two terms fewer each (tests/test_math.py re-derives the coefficients and
// checks the error).  Used by the LMPC kernel (+1 % on C5) and for PMPC's cosine at the iterate
// (+0.4 % on C2); PMPC's line-search sincos and RMPC keep the Taylor form, which their register
// allocation prefers (A/B: -0.6 % / -0.4 % with this one).
#define DART_SIN_COEFFS -0.16666666666666663, 0.00833333333333285, -0.0001984126984096554, 2.755731912250289e-06, \
                        -2.505208918178363e-08, 1.6056973209300557e-10, -7.52855132478024e-13
#define DART_COS_COEFFS -0.5, 0.041666666666666664, -0.0013888888888888367, 2.480158730131862e-05, \
                        -2.7557319146330464e-07, 2.087674380080511e-09, -1.1469439869437463e-11, 4.709676860456087e-14
__device__ __forceinline__ double sin_poly_(double y) {      // (sin x - x) / x^3 as a polynomial in y = x^2
    constexpr double c[7] = {DART_SIN_COEFFS};
    double p = c[6];
#pragma unroll
    for (int i = 5; i >= 0; --i) p = fma(p, y, c[i]);
    return p;
}
__device__ __forceinline__ double cos_poly_(double y) {      // (cos x - 1) / x^2 as a polynomial in y = x^2
    constexpr double c[8] = {DART_COS_COEFFS};
    double p = c[7];
#pragma unroll
    for (int i = 6; i >= 0; --i) p = fma(p, y, c[i]);
    return p;
}
__device__ __forceinline__ void sincos_econ(double x, double& s, double& c) {
    const double y = x * x;
    s = fma(x * y, sin_poly_(y), x);
    c = fma(y, cos_poly_(y), 1.0);
}
__device__ __forceinline__ double cos_econ(double x) {       // the cosine half of sincos_econ
    const double y = x * x;
    return fma(y, cos_poly_(y), 1.0);
}
// poly: |bounds| <= 1 rad (every configuration of the reference); the library branch is laid out off
// the hot path (PMPC: C2 +2.1 %, N = 15 +5.9 %, A/B tools/ab_lib.sh)
__device__ __forceinline__ double tilt_cos(bool poly, double x) {
    if (__builtin_expect(poly, 1)) return cos_small(x);
    return cos(x);
}
__device__ __forceinline__ void tilt_sincos(bool poly, double x, double& s, double& c) {
    if (__builtin_expect(poly, 1)) sincos_small(x, s, c);
    else sincos(x, &s, &c);
}
__device__ __forceinline__ double tilt_cos_econ(bool poly, double x) {
    if (__builtin_expect(poly, 1)) return cos_econ(x);
    return cos(x);
}
// (no layout hint here: RMPC measured 0.8 % slower with it, its register allocation moved)
__device__ __forceinline__ void tilt_sincos_econ(bool poly, double x, double& s, double& c) {
    if (poly) sincos_econ(x, s, c);
    else sincos(x, &s, &c);
}

// exp / tanh (LMPC, RMPC) by Cody-Waite reduction to |r| <= ln2/2 and P(r) = (e^r - 1 - r) / r^2 as the
// degree-19 Taylor polynomial economised by Chebyshev polynomials on |r| <= 0.3467 to degree 10 (one term
// fewer than the degree-11 Taylor P the kernels used before; the same 0.99 ulp for exp and 1.08 ulp for
// expm1 in double, tests/test_math.py).  tanh(x) = em / (em + 2), em = expm1(2x); exp underflows to the
// subnormals and 0 like libm.
#define DART_EXPM1_COEFFS 0.5, 0.1666666666666667, 0.04166666666666668, 0.008333333333326119, \
                          0.0013888888888879054, 0.0001984126987487566, 2.4801587336499025e-05, \
                          2.7557255330683724e-06, 2.755726321849137e-07, 2.5105245845597674e-08, 2.0918160101597142e-09
__device__ __forceinline__ double expm1_poly_(double r) {
    constexpr double c[11] = {DART_EXPM1_COEFFS};
    double p = c[10];
#pragma unroll
    for (int i = 9; i >= 0; --i) p = fma(p, r, c[i]);
    return p;
}
__device__ __forceinline__ double tanh_econ(double x) {
    const double y = fmin(fmax(2.0 * x, -80.0), 80.0);
    const double n = __builtin_rint(y * 1.4426950408889634);
    double r = fma(-n, 6.93147180369123816490e-01, y);
    r = fma(-n, 1.90821492927058770002e-10, r);
    const double q = fma(expm1_poly_(r) * r, r, r);
    const double sc = __builtin_ldexp(1.0, (int)n);
    const double em = fma(sc, q, sc - 1.0);
    return em * frcp(em + 2.0);
}
__device__ __forceinline__ double exp_econ(double x) {
    const double y = fmin(fmax(x, -745.0), 709.0);
    const double n = __builtin_rint(y * 1.4426950408889634);
    double r = fma(-n, 6.93147180369123816490e-01, y);
    r = fma(-n, 1.90821492927058770002e-10, r);
    double p = expm1_poly_(r);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    const int ni = (int)n, n1 = ni / 2, n2 = ni - n1;
    return __builtin_ldexp(__builtin_ldexp(p, n1), n2);
}

// natural log of x = m 2^e (m = frexp mantissa in [0.5, 1)), fdlibm's e_log.c reduction and
// minimax polynomial (Lg1..Lg7, < 1 ulp): 1 + f in [sqrt(2)/2, sqrt(2)), s = f / (2 + f),
// log(1 + f) = f - (hfsq - s (hfsq + R(s^2))).  Shared by the device log_fast and its host check
// (tools/check_log.cpp); rcp2f(f) supplies 1 / (2 + f).
template <class Rcp>
__host__ __device__ __forceinline__ double log_core(double m, int e, Rcp rcp2f) {
    if (m < 0.70710678118654752440) { m *= 2.0; e -= 1; }
    const double f = m - 1.0, k = (double)e;
    const double s = f * rcp2f(f), z = s * s, w = z * z;
    const double t1 = w * fma(w, fma(w, 1.531383769920937332e-01, 2.222219843214978396e-01), 3.999999999940941908e-01);
    const double t2 = z * fma(w, fma(w, fma(w, 1.479819860511658591e-01, 1.818357216161805012e-01),
                                     2.857142874366239149e-01), 6.666666666666735130e-01);
    const double R = t2 + t1, hfsq = 0.5 * f * f;
    return k * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + k * 1.90821492927058770002e-10)) - f);
}
struct RcpTwoPlus {     // 1 / (2 + f) for f in [-0.3, 0.42]: v_rcp_f64 + one Newton step
    __device__ double operator()(double f) const { return frcp(2.0 + f); }
};
// log for the barrier terms (positive normal arguments; NaN for x <= 0 or non-finite x, so a
// trial outside the box is rejected by the filter like with the library log).  About half the
// instructions of the library log; < 1 ulp (host check).
__device__ __forceinline__ double log_fast(double x) {
    const double m = __builtin_amdgcn_frexp_mant(x);
    const int e = __builtin_amdgcn_frexp_exp(x);
    const double r = log_core(m, e, RcpTwoPlus());
    return (x > 0.0 && x < 1.0e308) ? r : __builtin_nan("");
}

// IPOPT's Compare_le: lhs <= rhs up to 10 machine epsilons of |base| (filter acceptance tests)
__device__ __forceinline__ bool cmp_le(double lhs, double rhs, double base) {
    return lhs - rhs <= 10.0 * 2.220446049250313e-16 * fabs(base);
}

}  // namespace dartmpc
