// stamps.h -- diagnostic per-phase cycle counters (s_memtime) for the DART_STAMPS build only.
// Each kernel TU defines its own __device__ array and flushes block 0's counters into it.
#pragma once

#ifdef DART_STAMPS
#define STAMP_DECL unsigned long long t_prev_ = __builtin_amdgcn_s_memtime(), t_acc_[32] = {0};
#define STAMP_ADD(i, n) do { t_acc_[i] += (unsigned long long)(n); } while (0)
#define STAMP(i) do { unsigned long long t_ = __builtin_amdgcn_s_memtime(); t_acc_[i] += t_ - t_prev_; t_prev_ = t_; } while (0)
#define STAMP_FLUSH_TO(arr, b) do { if ((b) == 0 && threadIdx.x == 0) for (int q_ = 0; q_ < 16; ++q_) arr[q_] = t_acc_[q_]; } while (0)
// nested interval timers (a sub-part of a phase): SPAN_BEGIN(v) ... SPAN_END(i, v) adds the cycles to slot i
#define SPAN_BEGIN(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define SPAN_END(i, v) do { t_acc_[i] += __builtin_amdgcn_s_memtime() - (v); } while (0)
#define STAMP_FLUSH32_TO(arr, b) do { if ((b) == 0 && threadIdx.x == 0) for (int q_ = 0; q_ < 32; ++q_) arr[q_] = t_acc_[q_]; } while (0)
#else
#define STAMP_DECL
#define STAMP_ADD(i, n) do {} while (0)
#define STAMP(i) do {} while (0)
#define STAMP_FLUSH_TO(arr, b) do {} while (0)
#define SPAN_BEGIN(v) do {} while (0)
#define SPAN_END(i, v) do {} while (0)
#define STAMP_FLUSH32_TO(arr, b) do {} while (0)
#endif
