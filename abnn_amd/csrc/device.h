// device.h -- device helpers shared by the kernels of the handle API
// (kernels.hip) and of the buffer-index launcher (raw.hip): the reference's
// per-event arithmetic (brain.metal:15-19,73-122) written operation for
// operation like the oracle (bit-identical fp32 under -ffp-contract=off),
// and wave-level primitives.
#pragma once

#include "engine.h"

#pragma clang fp contract(off)

namespace abnn {
namespace {

// rand01, brain.metal:15-19.
__device__ __forceinline__ float rand01(uint32_t s)
{
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return (float)(s & 0xFFFFFFu) * (1.0f / 16777216.0f);
}

// Age of a timestamp: lastF and clock are `uint` in the reference
// (brain.metal:43,45), so `now - ts` (brain.metal:74,80,116) wraps at 2^32.
// Timestamps are stored as u64 (README lastFiredNS); every decision takes the
// low 32 bits, so a stamp ahead of the clock ages like the reference's.
__device__ __forceinline__ uint32_t age32(uint64_t now, uint64_t ts) { return (uint32_t)now - (uint32_t)ts; }

// Metal clamp(x, lo, hi) = min(max(x, lo), hi), written as selects so the
// result is bit-identical to the C oracle (no NaN canonicalisation).
__device__ __forceinline__ float clampf(float x, float lo, float hi)
{
    float m = x > lo ? x : lo;
    return m < hi ? m : hi;
}

__device__ __forceinline__ bool spike_candidate(const KernelParams& kp, float w, uint64_t tg,
                                                uint64_t now)
{
    float prob = clampf((w * w) * kp.base_scale, 0.0f, 1.0f);      // brain.metal:91
    return prob > rand01((uint32_t)tg ^ (uint32_t)now);             // brain.metal:92
}

__device__ __forceinline__ float updated_weight(const KernelParams& kp, float w, bool fired,
                                                float R, float rb, float isi)
{
    float dW = fired ? kp.a_ltp * (1.0f - w) : (-kp.a_ltd) * w;     // brain.metal:101-102
    dW = dW + (kp.eta_reward * (R - rb)) * (fired ? 1.0f : 0.0f);   // brain.metal:105-107
    float est_hz = isi > 0.0f ? 1e6f / isi : 0.0f;                  // brain.metal:116-117
    dW = dW + (kp.eta_home * (kp.target_rate_hz - est_hz)) * w;     // brain.metal:118
    return clampf(w + dW, kp.w_min, kp.w_max);                      // brain.metal:121
}

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t wave_uniform(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// A wave-uniform READ through the scalar data cache (s_load, counted by
// lgkmcnt): the gate's prologue reads its range bounds and the pass-start
// scalars this way, so they do not queue behind the filter's LDS-DMA and the
// first record loads, which vmcnt counts in issue order.  Only for values no
// wave of the launch writes before every wave has read them (the previous
// launch or the host wrote them).  Never a write: nothing stores through the
// scalar cache.
template <typename T>
__device__ __forceinline__ T sload(const T* p)
{
    return *(const __attribute__((address_space(4))) T*)p;
}

// Inclusive wave scan on DPP (row_shr within 16-lane rows, then the gfx9
// row broadcasts): six VALU ops, no LDS crossbar round trips.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x)
{
    int v = (int)x;
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return (uint32_t)v;
}

}  // namespace
}  // namespace abnn
