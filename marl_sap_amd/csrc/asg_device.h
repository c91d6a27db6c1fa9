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

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
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

// purposes of Philox counters (counter.z); counter.w = episode
enum : uint32_t { kCtrScale = 1u, kCtrPair = 2u, kCtrSpread = 3u, kCtrPerm = 4u, kCtrAction = 5u };

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
// generate_benefits_over_time, mock_constellation_env.py:281-293).
struct Bump {
    double scale;   // 0 when the pair is inactive
    double center;
    double s2;
};

__device__ __forceinline__ Bump philox_bump(EnvKey key, uint32_t episode, int i, int j, int m,
                                            int T, double wmin, double wmax, bool dense) {
    const u32x4 sc = philox4x32_10(u32x4{(uint32_t)j, 0u, kCtrScale, episode}, key.k0, key.k1);
    const double scale = (sc.x & 3u) == 3u ? 10.0 : 1.0;  // choice([1, 1, 1, 10])
    const uint32_t pair = (uint32_t)(i * m + j);
    const u32x4 a = philox4x32_10(u32x4{pair, 0u, kCtrPair, episode}, key.k0, key.k1);
    const bool active = dense || (u01_53(a.x, a.y) > 0.75);
    Bump b;
    b.scale = active ? scale : 0.0;
    b.center = 0.0 + (double)T * u01_53(a.z, a.w);
    const u32x4 s = philox4x32_10(u32x4{pair, 0u, kCtrSpread, episode}, key.k0, key.k1);
    b.s2 = bump_s2(wmin + (wmax - wmin) * u01_53(s.x, s.y));
    return b;
}

__device__ __forceinline__ double bump_at(const Bump &b, int t) {
    return b.scale == 0.0 ? 0.0 : bump_value(b.scale, b.center, b.s2, t);
}

// ---------------------------------------------------------------------------------
// wave64 reductions (ds_swizzle/DPP via __shfl_xor)
// ---------------------------------------------------------------------------------
__device__ __forceinline__ double wave_min_f64(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmin(v, __shfl_xor(v, o, kWave));
    return v;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint64_t w = __shfl_xor(v, o, kWave);
        v = w > v ? w : v;
    }
    return v;
}
__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, kWave));
    return v;
}
__device__ __forceinline__ int wave_or_i32(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v |= __shfl_xor(v, o, kWave);
    return v;
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
