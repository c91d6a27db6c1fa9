// asg_device.h -- device helpers shared by the env and LSA kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/asg.h"

namespace asg {

constexpr int kWave = 64;

// ---------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11): counter-based, so every (env, episode, pair)
// draw is a pure function of its key -- no RNG state in HBM, identical on any rank.
// ---------------------------------------------------------------------------------
struct u32x4 {
    uint32_t x, y, z, w;
};

#ifndef ASG_PHILOX_MAD64
#define ASG_PHILOX_MAD64 1
#endif
#ifndef ASG_PHILOX_BITOP3
#define ASG_PHILOX_BITOP3 1
#endif
__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
#if ASG_PHILOX_MAD64
        // one v_mad_u64_u32 per product instead of v_mul_hi_u32 + v_mul_lo_u32
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
#else
        const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
#endif
#if ASG_PHILOX_BITOP3
        // three-input XOR in one v_bitop3_b32 (truth table 0x96; gfx950)
        c = u32x4{(uint32_t)__builtin_amdgcn_bitop3_b32(hi1, c.y, k0, 0x96), lo1,
                  (uint32_t)__builtin_amdgcn_bitop3_b32(hi0, c.w, k1, 0x96), lo0};
#else
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
#endif
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// numpy's random_sample construction from two 32-bit words: 53-bit double in [0, 1)
__device__ __forceinline__ double u01_53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// np.log(0.05) as numpy rounds it (mock_constellation_env.py:293)
constexpr double kLog005 = -0x1.7f7427b73e391p+1;

// sigma_2 of mock_constellation_env.py:293 (sic: a sqrt named sigma_2)
__device__ __forceinline__ double bump_s2(double spread) {
    return sqrt(spread * spread / -8.0 / kLog005);
}

// benefit of one bump at time t (mock_constellation_env.py:298), same operation order
__device__ __forceinline__ double bump_value(double scale, double center, double s2, int t) {
    const double x = (double)t - center;
    return scale * exp(-(x * x) / s2 * 0.5);  // "/ 2" is exact as "* 0.5"
}

// the table entry B[t] of one recorded MT19937 bump p = (center, +-spread; scale 10 as a negative
// spread, (0, 0) for no bump): every reader of the compat-mode benefits evaluates it through
// this one function, so the float32 table written at reset and the float64 values evaluated
// later agree bit for bit
__device__ __forceinline__ double mt_par_value(double2 p, int t) {
    if (p.y == 0.0) return 0.0;
    return bump_value(p.y < 0.0 ? 10.0 : 1.0, p.x, bump_s2(__builtin_fabs(p.y)), t);
}

// purposes of Philox counters (counter.z); counter.w = episode
enum : uint32_t { kCtrScale = 1u, kCtrPair = 2u, kCtrSpread = 3u, kCtrPerm = 4u, kCtrAction = 5u, kCtrSelect = 6u,
                  kCtrSapNoise = 7u, kCtrPair2 = 8u, kCtrPair4 = 9u, kCtrBidsNoise = 10u };

// "a beats b" in torch.max order: NaN wins, then larger value, then smaller index.
// Branch-free (bitwise on the predicates) so it lowers to compares + v_cndmask.
__device__ __forceinline__ bool better(float va, int ja, float vb, int jb) {
    const bool na = va != va, nb = vb != vb, lt = ja < jb;
    return (na & (!nb | lt)) | (!nb & ((va > vb) | ((va == vb) & lt)));
}

// Key of one env's stream: seed and global env index (a 1-GPU run and an
// 8-GPU run of the same global indices draw identical benefits).
struct EnvKey {
    uint32_t k0, k1;
};
__device__ __forceinline__ EnvKey env_key(uint64_t seed, int64_t global_env) {
    return EnvKey{(uint32_t)seed ^ (uint32_t)((uint64_t)global_env >> 32) * 0x85EBCA6Bu,
                  (uint32_t)(seed >> 32) ^ (uint32_t)global_env};
}

// Bump parameters of one (agent i, task j) pair under Philox (the distribution of
// generate_benefits_over_time, mock_constellation_env.py:281-293): active with probability
// 0.25 (rand() > 0.75), center ~ U(0, T), width ~ U(wmin, wmax),
// sigma_2 = sqrt(w^2 / -8 / ln 0.05), value(t) = scale * exp(-(t - c)^2 / sigma_2 / 2)
// = scale * 2^(-(t - c)^2 * a2) with a2 = log2(e) / (2 sigma_2).  One Philox call serves
// four pairs (one 32-bit word each); the per-task scale (choice([1,1,1,10])) is a per-task
// draw.  The parameters are float32 values; the center is drawn on a grid of 2^-q with
// q = 24 - bits(T), so t - center is exact in float32 for every integer t < T.
struct Bump32 {
    float scale;  // 0 when the pair is inactive
    float center;
    float a2;     // log2(e) / (2 sigma_2)
};

__device__ __forceinline__ float philox_task_scale(EnvKey key, uint32_t episode, int j) {
    const u32x4 sc = philox4x32_10(u32x4{(uint32_t)j, 0u, kCtrScale, episode}, key.k0, key.k1);
    return (sc.x & 3u) == 3u ? 10.0f : 1.0f;
}

// the bump-shape constants of one launch (T's center grid exponent q, the width range)
struct BumpShape {
    int T, q;
    float wmin, wspan14;  // wspan14 = (wmax - wmin) 2^-14 (exact: a power-of-two scale)
    float cscale;  // T * 2^-16: the center directly from the 16-bit draw when q >= 16 (T < 256)
};
__host__ __device__ inline BumpShape bump_shape(int T, float wmin, float wmax) {
    int bits = 0;
    for (unsigned t = (unsigned)(T > 0 ? T : 1); t; t >>= 1) ++bits;
    return BumpShape{T, 24 - bits, wmin, (wmax - wmin) * 0x1p-14f, (float)T * 0x1p-16f};
}

// Pair 4k + s takes word s of Philox call k (counter {k, 0, kCtrPair4, episode}):
//   center = T * u16 on the 2^-q grid, u16 = w[31:16] * 2^-16: floor(u16 T 2^q) 2^-q
//   width  = wmin + (wmax - wmin) * w[15:2] * 2^-14
//   active = w[1:0] == 3 (probability 1/4)
// (42 bits of entropy per pair are plenty for a bump; one Philox call per four pairs halves
// the generator's share of the fused rollout's VALU against one per two pairs.)
__device__ __forceinline__ Bump32 bump_from_word(uint32_t w, float scale, const BumpShape &bs, bool dense) {
    Bump32 b;
    b.scale = (dense || (w & 3u) == 3u) ? scale : 0.0f;
    // the grid index (w >> 16) * T * 2^q / 2^16 is < T * 2^q <= 2^24: the 32-bit convert is exact;
    // for q >= 16 no bit is dropped and the center is (w >> 16) * T * 2^-16 exactly (a
    // product < 2^24 of an integer and a power of two): one convert and one multiply
    if (bs.q >= 16)
        b.center = (float)(w >> 16) * bs.cscale;
    else
        b.center = __builtin_ldexpf(
            (float)(uint32_t)((((uint64_t)(w >> 16) * (uint64_t)(uint32_t)bs.T) << bs.q) >> 16), -bs.q);
    // wmin + wspan u14 2^-14: (wspan 2^-14) u14 is the same exact product, one multiply fewer
    const float spread = bs.wmin + bs.wspan14 * (float)((w >> 2) & 0x3fffu);
    // log2(e) / (2 sigma_2), sigma_2 = sqrt(spread^2 / -8 / ln 0.05), is for spread > 0
    // log2(e) sqrt(-2 ln 0.05) / spread: one v_rcp_f32 (<= 1 ulp) and a multiply (within
    // 3e-7 relative of the float64 formula; parity checks use the exported parameters)
    b.a2 = 0x1.c4035ap+1f * __builtin_amdgcn_rcpf(spread);
    return b;
}
// pairs pair0 .. pair0 + 3 (pair0 % 4 == 0): one Philox call
__device__ __forceinline__ void philox_bump32x4(EnvKey key, uint32_t episode, int pair0, const float (&scale)[4],
                                                const BumpShape &bs, bool dense, Bump32 (&b)[4]) {
    const u32x4 r = philox4x32_10(u32x4{(uint32_t)pair0 >> 2, 0u, kCtrPair4, episode}, key.k0, key.k1);
    b[0] = bump_from_word(r.x, scale[0], bs, dense);
    b[1] = bump_from_word(r.y, scale[1], bs, dense);
    b[2] = bump_from_word(r.z, scale[2], bs, dense);
    b[3] = bump_from_word(r.w, scale[3], bs, dense);
}
__device__ __forceinline__ Bump32 philox_bump32(EnvKey key, uint32_t episode, int pair, float scale,
                                                const BumpShape &bs, bool dense) {
    const u32x4 r = philox4x32_10(u32x4{(uint32_t)pair >> 2, 0u, kCtrPair4, episode}, key.k0, key.k1);
    const int s = pair & 3;
    const uint32_t w = s == 0 ? r.x : (s == 1 ? r.y : (s == 2 ? r.z : r.w));
    return bump_from_word(w, scale, bs, dense);
}

__device__ __forceinline__ Bump32 philox_bump32(EnvKey key, uint32_t episode, int pair, float scale, int T,
                                                float wmin, float wmax, bool dense) {
    return philox_bump32(key, episode, pair, scale, bump_shape(T, wmin, wmax), dense);
}

// float32 evaluation: value(t) = scale * 2^(-(x * x) * a2), x = t - center exact (the center
// is on the 2^-q grid); the exponent y = x^2 a2 carries two float32 roundings, so the relative
// error is <= y ln2 2^-23 + 1.5 2^-23 and the absolute error <= 1.5 2^-23 scale at every y (the
// bump's peak height in float32 ulps); relative <= 1e-6 wherever y <= 12 (values >= 2^-12
// scale).  v_exp_f32 flushes results below FLT_MIN to 0.  (Rounds 1-4 carried y as a double-
// float pair -- relative 1e-6 at every y -- in 9 VALU instead of 4 per value: 96 values per
// 32-row tile-pass made it 10 % of the episode kernel's VALU; this form is 4 % faster per step,
// r5 A/B.)  Rewards and the `beta > 1e-12` mask use the float64 evaluation (bump64_at).
__device__ __forceinline__ float bump32_at(const Bump32 &b, int t) {
    const float x = (float)t - b.center;
    return b.scale * __builtin_amdgcn_exp2f(-(x * x) * b.a2);
}

// The same bump in float64 (the reference's arithmetic, mock :293, on these parameters).
// Used where a value is compared or accumulated in float64 -- the reward's beta_hat and its
// `beta > 1e-12` mask (n values per step) -- and by the table export.
__device__ __forceinline__ double bump64_at(const Bump32 &b, int t) {
    const double x = (double)t - (double)b.center;
    return (double)b.scale * exp2(-(x * x) * (double)b.a2);
}

// ---------------------------------------------------------------------------------
// wave64 butterflies on the VALU: DPP inside 16-lane rows (quad xor 1, quad xor 2,
// half-row mirror, row mirror), then v_permlane16_swap / v_permlane32_swap across rows
// (gfx950).  Every lane ends with the full reduction.  Call in wave-uniform control flow.
// ---------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
// v_permlane{16,32}_swap with both operands = x: element 0 / element 1 of the result
// hold this lane's and the partner lane's value (lane ^ 16 / lane ^ 32), in an order
// that depends on the lane -- reductions combine both, so the order never matters.
struct SwapPair {
    uint32_t a, b;
};
__device__ __forceinline__ SwapPair swap16(uint32_t x) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return SwapPair{r[0], r[1]};
}
__device__ __forceinline__ SwapPair swap32(uint32_t x) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return SwapPair{r[0], r[1]};
}

template <class T, class Op>
__device__ __forceinline__ T wave_allreduce(T v, Op op) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32/64-bit values");
    auto dstep = [&](auto perm) {  // DPP: partner value from a lane permutation
        if constexpr (sizeof(T) == 4) {
            v = op(v, __builtin_bit_cast(T, perm(__builtin_bit_cast(uint32_t, v))));
        } else {
            const uint64_t x = __builtin_bit_cast(uint64_t, v);
            const uint64_t y = (uint64_t)perm((uint32_t)x) | ((uint64_t)perm((uint32_t)(x >> 32)) << 32);
            v = op(v, __builtin_bit_cast(T, y));
        }
    };
    auto sstep = [&](auto swp) {   // permlane swap: combine both halves of the pair
        if constexpr (sizeof(T) == 4) {
            const SwapPair p = swp(__builtin_bit_cast(uint32_t, v));
            v = op(__builtin_bit_cast(T, p.a), __builtin_bit_cast(T, p.b));
        } else {
            const uint64_t x = __builtin_bit_cast(uint64_t, v);
            const SwapPair lo = swp((uint32_t)x), hi = swp((uint32_t)(x >> 32));
            v = op(__builtin_bit_cast(T, (uint64_t)lo.a | ((uint64_t)hi.a << 32)),
                   __builtin_bit_cast(T, (uint64_t)lo.b | ((uint64_t)hi.b << 32)));
        }
    };
    dstep([](uint32_t x) { return dpp32<0xB1>(x); });   // quad_perm [1,0,3,2]
    dstep([](uint32_t x) { return dpp32<0x4E>(x); });   // quad_perm [2,3,0,1]
    dstep([](uint32_t x) { return dpp32<0x141>(x); });  // row_half_mirror
    dstep([](uint32_t x) { return dpp32<0x140>(x); });  // row_mirror
    sstep([](uint32_t x) { return swap16(x); });
    sstep([](uint32_t x) { return swap32(x); });
    return v;
}

__device__ __forceinline__ double wave_min_f64(double v) {
    return wave_allreduce(v, [](double a, double b) { return fmin(a, b); });
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
    return wave_allreduce(v, [](uint64_t a, uint64_t b) { return a > b ? a : b; });
}
__device__ __forceinline__ int wave_max_i32(int v) {
    return wave_allreduce(v, [](int a, int b) { return a > b ? a : b; });
}
__device__ __forceinline__ int wave_or_i32(int v) {
    return wave_allreduce(v, [](int a, int b) { return a | b; });
}

// wave64 minimum of a float32 that is never NaN, returned wave-uniform (SGPR): one block
// of DPP-fused v_min_f32 (fminf on DPP operands would add a canonicalising v_max per
// step) -- 4 steps inside each 16-lane row, then row_bcast:15 / row_bcast:31 fold the rows
// into lane 63.  s_nop 1 covers the VALU-write -> DPP-read hazard.  Call in wave-uniform
// control flow.
__device__ __forceinline__ float wave_min_f32_nonan(float x0) {
#ifndef ASG_LSA_PERMLANE_MIN
    float x;  // a separate result register: the input stays live without a copy
    asm("s_nop 1\n\t"
        "v_min_f32_dpp %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc"
        : "=&v"(x)
        : "v"(x0));
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 63));
#else
    const float x = x0;
    float y, t;
    asm("s_nop 1\n\t"
        "v_min_f32_dpp %0, %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32 %1, %0\n\t"
        "s_nop 1\n\t"
        "v_permlane16_swap_b32 %0, %1\n\t"
        "v_min_f32 %0, %0, %1\n\t"
        "v_mov_b32 %1, %0\n\t"
        "s_nop 1\n\t"
        "v_permlane32_swap_b32 %0, %1\n\t"
        "v_min_f32 %0, %0, %1"
        : "=&v"(y), "=&v"(t)
        : "v"(x));
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, y)));
#endif
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    return wave_allreduce(v, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
}
// wave64 maximum of a uint32, returned wave-uniform: the row_bcast fold of
// wave_min_f32_nonan with v_max_u32
__device__ __forceinline__ uint32_t wave_max_u32_bcast(uint32_t x) {
    asm("s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc"
        : "+v"(x));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// wave64 maximum of a float32 that is never NaN, returned wave-uniform: the row_bcast
// fold of wave_min_f32_nonan with v_max_f32
__device__ __forceinline__ float wave_max_f32_nonan(float x) {
    asm("s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc"
        : "+v"(x));
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 63));
}

// uniform read of a lane-distributed register array: element idx lives in lane idx % 64,
// slot idx / 64 (idx wave-uniform)
// (one v_readlane per slot, then scalar selects: the compiler must not turn the slot pick
// into a dynamically indexed private array, which would live in scratch)
template <int N, class T>
__device__ __forceinline__ T lane_get(const T (&x)[N], int idx) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32/64-bit values");
    const int slot = idx >> 6, src = idx & 63;
    if constexpr (sizeof(T) == 4) {
        int sel = __builtin_amdgcn_readlane(__builtin_bit_cast(int, x[0]), src);
#pragma unroll
        for (int c = 1; c < N; ++c) {
            const int t = __builtin_amdgcn_readlane(__builtin_bit_cast(int, x[c]), src);
            sel = (c == slot) ? t : sel;
        }
        return __builtin_bit_cast(T, sel);
    } else {
        uint64_t sel = 0;
#pragma unroll
        for (int c = 0; c < N; ++c) {
            const uint64_t u = __builtin_bit_cast(uint64_t, x[c]);
            const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)u, src);
            const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), src);
            const uint64_t t = (uint64_t)lo | ((uint64_t)hi << 32);
            sel = (c == 0 || c == slot) ? t : sel;
        }
        return __builtin_bit_cast(T, sel);
    }
}
template <int N, class T>
__device__ __forceinline__ void lane_set(T (&x)[N], int idx, T val) {
    const int slot = idx >> 6, dst = idx & 63;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < N; ++c) x[c] = (c == slot && lane == dst) ? val : x[c];
}

// wave-scope barrier with LDS/global ordering (a workgroup may hold other waves that do
// not take part, so __syncthreads is not usable inside per-wave code)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// element pointer of a strided batch field
template <typename T>
__device__ __forceinline__ T *fptr(const asg_field &f, int64_t b, int64_t t, int64_t d2, int64_t d3) {
    return reinterpret_cast<T *>(f.ptr) + b * f.stride[0] + t * f.stride[1] + d2 * f.stride[2] +
           d3 * f.stride[3];
}

}  // namespace asg
