// sap_stage.h -- the SequentialAssignmentProblemSelector of one env on one wave64 (sap_selectors.py:
// 52-98, n <= m <= 64): its noisy Q column staged in registers (sap_stage), the certified fast path
// (optionally warm-started) with the scipy-exact solver behind it, the actions out (sap_emit).
// sap_select_kernel (asg_lsa.hip) runs one per wave; the same function called by the rollout
// kernel's Q-output waves after their env's Q rows measured slower.
#pragma once
#include "asg_device.h"
#include "lsa_wave.h"

namespace asg {

// square SAP problems (n == m) first take the certified fast path (lsa_fast_reg64: column
// reduction + shortest augmenting paths, used under a uniqueness certificate), the rest and
// every uncertified problem the scipy-exact solver; -DASG_SAP_FAST=0: the exact solver only
#ifndef ASG_SAP_FAST
#define ASG_SAP_FAST 1
#endif
#ifndef ASG_SAP_PIN
#define ASG_SAP_PIN 1
#endif
#ifndef ASG_SAP_PIN_BASE
#define ASG_SAP_PIN_BASE 32
#endif

// problem b's working column: Q column `lane` of env b plus its noise (std mean|Q| * eps * 2),
// negated (maximize) -- ASG_E_LSA_INVALID (wave uniform) when the noisy matrix holds NaN or
// +inf
template <bool kDense64, class RC>
__device__ __forceinline__ int sap_stage(const float *q, int64_t q0, int64_t q1, int64_t q2, int n, int m,
                                         float epsilon, uint64_t seed, uint32_t counter, int64_t env_base, int64_t b,
                                         RC &rc) {
    const int lane = threadIdx.x & (kWave - 1);
    float asum = 0.0f;
    if constexpr (kDense64) {
        // 64 x 64 rows of 64 contiguous floats (the rollout's Q rows): every lane and row valid,
        // the rows at compile-time offsets -- 64 loads off four base addresses, no guards
        const float *col = q + b * q0 + lane;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const float x = col[i * 64], y = col[(i + 32) * 64];
            asum += __builtin_fabsf(x);
            asum += __builtin_fabsf(y);
            rc.lo[i] = x;
            rc.hi[i] = y;
        }
    } else {
        // opaque strides: the 64 row offsets i * q1 are formed where used, not kept live
        asm volatile("" : "+s"(q0), "+s"(q1), "+s"(q2));
        const float *col = q + b * q0 + (int64_t)lane * q2;
        // in place in the column's registers
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            float x = 0.0f, y = 0.0f;
            if (lane < m && i < n) x = col[i * q1];
            if (lane < m && i + 32 < n) y = col[(i + 32) * q1];
            asum += __builtin_fabsf(x);
            asum += __builtin_fabsf(y);
            rc.lo[i] = x;
            rc.hi[i] = y;
        }
    }
    // th.mean(th.abs(Q)) (float32; summation order differs from torch's, the noise is
    // random either way), stds = avg * eps * 2
    const float avg = wave_allreduce(asum, [](float x, float y) { return x + y; }) / (float)(n * m);
    const float stdv = avg * epsilon * 2.0f;
    if (epsilon > 0.0f) {
        const EnvKey key = env_key(seed, env_base + b);
        constexpr float k2m24 = 5.9604644775390625e-08f;  // 2^-24
        constexpr float k2pi = 6.283185307179586f;
#pragma unroll
        for (int i4 = 0; i4 < 16; ++i4) {  // rows 4*i4 .. 4*i4+3 of this column
            const u32x4 r = philox4x32_10(u32x4{(uint32_t)lane, (uint32_t)i4, kCtrSapNoise, counter}, key.k0, key.k1);
            const float u1a = (float)((r.x >> 8) + 1u) * k2m24, u2a = (float)(r.y >> 8) * k2m24;
            const float u1b = (float)((r.z >> 8) + 1u) * k2m24, u2b = (float)(r.w >> 8) * k2m24;
            const float ra = __builtin_sqrtf(-2.0f * __logf(u1a)), rb = __builtin_sqrtf(-2.0f * __logf(u1b));
            const float z[4] = {ra * __cosf(k2pi * u2a), ra * __sinf(k2pi * u2a), rb * __cosf(k2pi * u2b),
                                rb * __sinf(k2pi * u2b)};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int i = 4 * i4 + k;  // torch.normal(0, std) = 0 + std * z, then Q += noise
                if (i < 32) rc.lo[i] = rc.lo[i] + stdv * z[k];
                else rc.hi[i - 32] = rc.hi[i - 32] + stdv * z[k];
            }
        }
    }
    int bad = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        // scipy on the noisy float64 matrix: NaN or +inf (-inf once negated) is invalid
        const bool va = lane < m && i < n, vb = lane < m && i + 32 < n;
        const float x = rc.lo[i], y = rc.hi[i];
        bad |= va & ((x != x) | (x == __builtin_inff()));
        bad |= vb & ((y != y) | (y == __builtin_inff()));
        rc.lo[i] = va ? -x : 0.0f;
        rc.hi[i] = vb ? -y : 0.0f;
    }
    // wave-uniform in the compiler's eyes too (slot state is updated under this branch)
    return __builtin_amdgcn_readfirstlane(wave_or_i32(bad)) ? ASG_E_LSA_INVALID : ASG_OK;
}

// one problem's outputs: the assignment as float32 actions (sap_selectors.py:91-97), or as
// the int64 the runner's batch.update casts them to (act_out: the EpisodeBatch actions row);
// -1 on error
template <bool kCount>
__device__ __forceinline__ void sap_emit(int64_t b, int status, int c4r, int steps, int n, int m, float *col_out,
                                         int64_t *act_out, int32_t *status_out, int32_t *steps_out) {
    const int lane = threadIdx.x & (kWave - 1);
    float *co = act_out ? nullptr : col_out + b * n;
    int64_t *ao = act_out ? act_out + b * n : nullptr;
    if (status == ASG_OK) {
        const int c[1] = {c4r};
        lsa_emit_wave(c, n, m, nullptr, nullptr, ao, co);
    } else {
        for (int i = lane; i < n; i += kWave) {
            if (ao) ao[i] = -1;
            else co[i] = -1.0f;
        }
    }
    if (kCount && lane == 0) steps_out[b] = steps;
    // asg_sap_select_into accumulates: the env's status word keeps its minimum over the episode's
    // calls (error codes are negative: the most negative code seen, not the first one), read once per episode instead of reduced after every call
    if (lane == 0 && status_out) status_out[b] = act_out ? min(status_out[b], status) : status;
}


// one env's selection: stage (noise of std 2 eps mean|Q|), fast path (kWarm: from `duals`, the
// env's column duals of its previous selection, NaN when the fast path did not finish, so the next
// call starts that env cold), the scipy-exact solver for the rest, the outputs.  slot: 64 u64 of
// LDS for this wave.  Wave-uniform arguments; all 64 lanes call it.
template <bool kCount, bool kDense64, bool kWarm>
__device__ __forceinline__ void sap_select_one(const float *q, int64_t q0, int64_t q1, int64_t q2, int n, int m,
                                               float epsilon, uint64_t seed, uint32_t counter, int64_t env_base,
                                               int64_t b, float *col_out, int64_t *act_out, int32_t *status_out,
                                               int32_t *steps_out, double *duals, int warm, uint64_t *slot) {
#if ASG_SAP_PIN
    RegColPin<ASG_SAP_PIN_BASE> rc;  // the column in v[BASE .. BASE + 63]: one indexed move per row read
#else
    RegCostF32 rc;
#endif
    int status = sap_stage<kDense64>(q, q0, q1, q2, n, m, epsilon, seed, counter, env_base, b, rc);
    int c4r[1] = {-1};
    int nsteps = 0, nfast = 0;
#ifdef ASG_SAP_STAGE_ONLY  // timing experiments only: the staging and noise alone (wrong results)
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < 32; ++k) sum += rc.lo[k] + rc.hi[k];
    if (__builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, sum)) == 0x7fffffff) status = 1;
    sap_emit<kCount>(b, status, (int)(threadIdx.x & 63), 0, n, m, col_out, act_out, status_out, steps_out);
    return;
#endif
    bool done = false;
    if constexpr (kWarm) {
        const int lane = threadIdx.x & 63;
        double *dp = duals + b * 64 + lane;
        const double vin = warm ? *dp : __builtin_nan("");
        double vnew = __builtin_nan("");
        if (ASG_SAP_FAST && status == ASG_OK && n == m)
            done = lsa_fast_reg64<decltype(rc), kCount, true>(rc, n, c4r, &nfast, slot, vin, &vnew) == ASG_OK;
        // only certified duals carry over: an env whose fast path ended uncertified (ties, NaN)
        // or did not run stores NaN and starts cold next call (lsa_fast_reg64 fills vnew before
        // its certificate)
        *dp = done ? vnew : __builtin_nan("");
    } else if (ASG_SAP_FAST && status == ASG_OK && n == m) {
        done = lsa_fast_reg64<decltype(rc), kCount>(rc, n, c4r, &nfast, slot) == ASG_OK;
    }
    if (status == ASG_OK && !done) status = lsa_solve_reg64<decltype(rc), kCount>(rc, n, m, c4r, &nsteps);
    // instrumented instance: fast-path steps in the low 16 bits, scipy-exact steps above
    sap_emit<kCount>(b, status, c4r[0], nfast | (nsteps << 16), n, m, col_out, act_out, status_out, steps_out);
}

}  // namespace asg
