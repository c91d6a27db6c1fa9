// asg_filtered.hip -- the filtered selectors of the real-env algorithms (gfx950).
//
// FilteredSAPActionSelector / FilteredEpsGrSAPTestActionSelector
// (action_selectors/filtered_sap_selectors.py:7-148) and FilteredEpsilonGreedyActionSelector /
// FilteredSoftPoliciesSelector (filtered_classic_selectors.py:6-103).  The agent emits M + 1
// Q-values per agent (its top-M tasks and a "do nothing else" baseline); the selectors map
// them onto the m tasks through each agent's top-M tasks by total benefit:
//   total[b][i][j]  = beta[b][i][j].sum(-1)                      (beta: float16 [B, n, m, L])
//   top[b][i]       = topk(total[b][i], M).indices                (descending)
//   mat[b][i][j]    = Q[b][i][M] + rand * 1e-8;  mat[b][i][top[s]] = Q[b][i][s]
// then LSA(maximize) per env (SAP; Gaussian noise of std 2 eps mean|mat[b]| first) or an
// epsilon-greedy argmax per row.  The reference loops over envs on the CPU (topk, indexing,
// scipy); here a wave per (env, agent) row does the L-sum + top-M selection and a wave per
// row writes the matrix, then the batched scipy-exact LSA (asg_lsa.hip) or the
// epsilon-greedy kernel (asg_select.hip, unmasked argmax) runs over all envs at once.
//
// Bit-parity: the L-sum is torch's (Half: float32 accumulation left to right, one rounding
// to half); the matrix entries are base + float32(u * 1e-8f) as torch rounds them; the
// tie noise u and the Gaussian noise can be given (the reference's draws) or drawn from
// Philox keyed by (seed, global env, counter).  torch.topk leaves the order of equal totals
// unspecified: here ties go to the lower index (tests pin tie-free inputs against the
// reference and the tie rule against the oracle).
#include <hip/hip_fp16.h>

#include "asg_device.h"
#include "asg_internal.h"

namespace asg {

enum : uint32_t { kCtrFiltTie = 8u, kCtrFiltGauss = 9u, kCtrFiltSoft = 10u };

// "a ranks before b" in torch.topk(largest) order: NaN first, then larger, then (our tie
// rule) the smaller index
template <class V>
__device__ __forceinline__ bool topk_before(V va, int ja, V vb, int jb) {
    const bool na = va != va, nb = vb != vb, lt = ja < jb;
    return (na & (!nb | lt)) | (!nb & ((va > vb) | ((va == vb) & lt)));
}

template <class V>
__device__ __forceinline__ V load_total(const void *beta, int dtype, int64_t off, int64_t sl, int L) {
    if (dtype == ASG_F16) {
        const __half *p = reinterpret_cast<const __half *>(beta) + off;
        float acc = 0.0f;
        for (int l = 0; l < L; ++l) acc = acc + __half2float(p[l * sl]);
        return (V)__half2float(__float2half(acc));  // torch's Half sum: one rounding to half
    }
    if (dtype == ASG_F32) {
        const float *p = reinterpret_cast<const float *>(beta) + off;
        float acc = 0.0f;
        for (int l = 0; l < L; ++l) acc = acc + p[l * sl];
        return (V)acc;
    }
    const double *p = reinterpret_cast<const double *>(beta) + off;
    double acc = 0.0;
    for (int l = 0; l < L; ++l) acc = acc + p[l * sl];
    return (V)acc;
}

// One wave per (env, agent) row: the L-summed totals of the row's m tasks, CAP per lane
// (task j = lane + 64 c), then M rounds of a wave arg-max with the picked task retired.
template <int CAP, class V>
__global__ void __launch_bounds__(256) filtered_topm_kernel(const void *beta, int dtype, int64_t s0, int64_t s1,
                                                            int64_t s2, int64_t s3, int64_t B, int n, int m, int L,
                                                            int M, int64_t *topm) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (row >= B * n) return;  // whole waves exit together
    const int64_t b = row / n;
    const int i = (int)(row - b * n);
    V v[CAP];
    uint32_t live = 0;
#pragma unroll
    for (int c = 0; c < CAP; ++c) {
        const int j = lane + 64 * c;
        if (j < m) {
            v[c] = load_total<V>(beta, dtype, b * s0 + (int64_t)i * s1 + (int64_t)j * s2, s3, L);
            live |= 1u << c;
        } else {
            v[c] = (V)0;
        }
    }
    for (int s = 0; s < M; ++s) {
        V bv = (V)0;
        int bj = 0x7fffffff;
#pragma unroll
        for (int c = 0; c < CAP; ++c) {
            const int j = lane + 64 * c;
            if (((live >> c) & 1u) && (bj == 0x7fffffff || topk_before<V>(v[c], j, bv, bj))) {
                bv = v[c];
                bj = j;
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const V ov = __shfl_xor(bv, o);
            const int oj = __shfl_xor(bj, o);
            if (oj != 0x7fffffff && (bj == 0x7fffffff || topk_before<V>(ov, oj, bv, bj))) {
                bv = ov;
                bj = oj;
            }
        }
        if ((bj & 63) == lane) live &= ~(1u << (bj >> 6));
        if (lane == 0) topm[row * M + s] = bj;
    }
}

// One wave per (env, agent) row: the row staged in LDS (base + tie noise, then the top-M
// Q-values scattered), written out coalesced; the row's sum |x| (float64) for the SAP
// noise scale.
__global__ void __launch_bounds__(256) filtered_matrix_kernel(const float *q, int64_t q0, int64_t q1, int64_t q2,
                                                              const int64_t *topm, int64_t B, int n, int m, int M,
                                                              const float *tie, uint64_t seed, uint32_t counter,
                                                              int64_t env_base,
                                                              float *mat, double *rowabs) {
    extern __shared__ float s_row[];  // [4][m]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t row = (int64_t)blockIdx.x * 4 + w;
    if (row >= B * n) return;
    const int64_t b = row / n;
    const int i = (int)(row - b * n);
    float *sr = s_row + (int64_t)w * m;
    const float *qr = q + b * q0 + (int64_t)i * q1;
    const float base = qr[(int64_t)M * q2];
    const EnvKey key = env_key(seed, env_base + b);
    constexpr float k2m24 = 5.9604644775390625e-08f;  // 2^-24: torch.rand's float32 grid
    const float scale = 1e-8f;                         // the reference's python 1e-8 as float32
    for (int j0 = 4 * lane; j0 < m; j0 += 256) {
        float u[4];
        if (tie) {
#pragma unroll
            for (int c = 0; c < 4; ++c) u[c] = j0 + c < m ? tie[row * m + j0 + c] : 0.f;
        } else {
            const u32x4 r = philox4x32_10(u32x4{(uint32_t)(j0 >> 2), (uint32_t)i, kCtrFiltTie, counter}, key.k0, key.k1);
            u[0] = (float)(r.x >> 8) * k2m24;
            u[1] = (float)(r.y >> 8) * k2m24;
            u[2] = (float)(r.z >> 8) * k2m24;
            u[3] = (float)(r.w >> 8) * k2m24;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float nz = u[c] * scale;
            if (j0 + c < m) sr[j0 + c] = base + nz;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    if (lane < M) sr[topm[row * M + lane]] = qr[(int64_t)lane * q2];
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
    double acc = 0.0;
    for (int j = lane; j < m; j += 64) {
        const float x = sr[j];
        mat[row * m + j] = x;
        acc += (double)__builtin_fabsf(x);
    }
    acc = wave_allreduce(acc, [](double a, double c) { return a + c; });
    if (lane == 0 && rowabs) rowabs[row] = acc;
}

// FilteredSAPActionSelector exploration: per env, std = float32(float32(mean|mat| * eps) * 2)
// and mat += N(0, std^2) (Philox Box-Muller), or mat += the given noise.  One workgroup per
// env.
// The per-row float64 sums of |mat| are formed here (a wave per row, lane j-strided then a
// wave sum: the association filtered_matrix_kernel uses) into LDS, so the selection needs no
// scratch buffer in HBM.
__global__ void __launch_bounds__(256) filtered_gauss_kernel(float *mat, int n, int m, float epsilon,
                                                             const float *gauss, uint64_t seed, uint32_t counter,
                                                             int64_t env_base) {
    __shared__ double s_part[4];
    extern __shared__ double s_rowabs[];  // [n]
    const int64_t b = blockIdx.x;
    const int64_t nm = (int64_t)n * m;
    float *mb = mat + b * nm;
    if (gauss) {
        const float *g = gauss + b * nm;
        for (int64_t x = threadIdx.x; x < nm; x += blockDim.x) mb[x] = mb[x] + g[x];
        return;
    }
    {
        const int lane = threadIdx.x & 63;
        for (int i = threadIdx.x >> 6; i < n; i += (int)(blockDim.x >> 6)) {
            double ra = 0.0;
            for (int j = lane; j < m; j += 64) ra += (double)__builtin_fabsf(mb[(int64_t)i * m + j]);
            ra = wave_allreduce(ra, [](double a, double c) { return a + c; });
            if (lane == 0) s_rowabs[i] = ra;
        }
    }
    __syncthreads();
    double acc = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) acc += s_rowabs[i];
    acc = wave_allreduce(acc, [](double a, double c) { return a + c; });
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = acc;
    __syncthreads();
    const double tot = s_part[0] + s_part[1] + s_part[2] + s_part[3];
    const float mean = (float)(tot / (double)nm);
    const float sd = (mean * epsilon) * 2.0f;
    const EnvKey key = env_key(seed, env_base + b);
    constexpr float k2m24 = 5.9604644775390625e-08f;
    constexpr float k2pi = 6.283185307179586f;
    for (int64_t x0 = 4 * (int64_t)threadIdx.x; x0 < nm; x0 += 4 * (int64_t)blockDim.x) {
        const u32x4 r = philox4x32_10(u32x4{(uint32_t)(x0 >> 2), (uint32_t)(x0 >> 34), kCtrFiltGauss, counter},
                                      key.k0, key.k1);
        const float u1a = (float)((r.x >> 8) + 1u) * k2m24, u2a = (float)(r.y >> 8) * k2m24;
        const float u1b = (float)((r.z >> 8) + 1u) * k2m24, u2b = (float)(r.w >> 8) * k2m24;
        const float ra = __builtin_sqrtf(-2.0f * __logf(u1a)), rb = __builtin_sqrtf(-2.0f * __logf(u1b));
        const float z[4] = {ra * __cosf(k2pi * u2a), ra * __sinf(k2pi * u2a), rb * __cosf(k2pi * u2b),
                            rb * __sinf(k2pi * u2b)};
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (x0 + c < nm) mb[x0 + c] = mb[x0 + c] + z[c] * sd;
    }
}

// FilteredSoftPoliciesSelector's mapping (filtered_classic_selectors.py:70-103): a picked
// index p < M is the agent's p-th top task; p == M is a uniformly random task outside the
// top M (the reference's argmax of uniforms with the top M masked).  One thread per row.
__global__ void filtered_soft_map_kernel(const int64_t *picked, const int64_t *topm, int64_t B, int n, int m, int M,
                                         uint64_t seed, uint32_t counter, int64_t env_base, int64_t *out, int *err) {
    const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= B * n) return;
    const int64_t p = picked[row];
    const int64_t *top = topm + row * M;
    if (p < 0 || p > M) {
        atomicCAS(err, 0, ASG_E_INVALID_ARG);
        out[row] = 0;
        return;
    }
    if (p < M) {
        out[row] = top[p];
        return;
    }
    const int64_t b = row / n;
    const int i = (int)(row - b * n);
    const EnvKey key = env_key(seed, env_base + b);
    const u32x4 r = philox4x32_10(u32x4{(uint32_t)i, 0u, kCtrFiltSoft, counter}, key.k0, key.k1);
    const int target = (int)(((uint64_t)r.x * (uint64_t)(m - M)) >> 32);  // in [0, m - M)
    // the target-th task (ascending) not in the top M: the fixed point j = target + #top <= j
    int j = target;
    for (int it = 0; it <= M; ++it) {
        int below = 0;
        for (int s = 0; s < M; ++s) below += top[s] <= j;
        const int nj = target + below;
        if (nj == j) break;
        j = nj;
    }
    out[row] = j;
}

static int cap_for(int m) {
    const int c = (m + 63) / 64;
    return c <= 1 ? 1 : c <= 2 ? 2 : c <= 4 ? 4 : c <= 8 ? 8 : c <= 16 ? 16 : 0;
}

hipError_t launch_filtered_topm(const void *beta, int dtype, const int64_t bs[4], int64_t B, int n, int m, int L, int M,
                                int64_t *topm, hipStream_t s) {
    const int64_t rows = B * n;
    const dim3 grid((unsigned)((rows + 3) / 4));
#define TOPM_(CAP, V)                                                                                            \
    hipLaunchKernelGGL((filtered_topm_kernel<CAP, V>), grid, dim3(256), 0, s, beta, dtype, bs[0], bs[1], bs[2], \
                       bs[3], B, n, m, L, M, topm)
#define TOPM_V(V)                  \
    switch (cap_for(m)) {          \
        case 1: TOPM_(1, V); break; \
        case 2: TOPM_(2, V); break; \
        case 4: TOPM_(4, V); break; \
        case 8: TOPM_(8, V); break; \
        default: TOPM_(16, V); break; \
    }
    if (dtype == ASG_F64) {
        TOPM_V(double)
    } else {
        TOPM_V(float)
    }
#undef TOPM_V
#undef TOPM_
    return hipGetLastError();
}

hipError_t launch_filtered_matrix(const float *q, const int64_t qs[3], const int64_t *topm, int64_t B, int n, int m,
                                  int M, const float *tie, uint64_t seed, uint32_t counter, int64_t env_base,
                                  float *mat, double *rowabs, hipStream_t s) {
    const int64_t rows = B * n;
    hipLaunchKernelGGL(filtered_matrix_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), sizeof(float) * 4 * m, s,
                       q, qs[0], qs[1], qs[2], topm, B, n, m, M, tie, seed, counter, env_base, mat, rowabs);
    return hipGetLastError();
}

hipError_t launch_filtered_gauss(float *mat, int64_t B, int n, int m, float epsilon, const float *gauss,
                                 uint64_t seed, uint32_t counter, int64_t env_base, hipStream_t s) {
    hipLaunchKernelGGL(filtered_gauss_kernel, dim3((unsigned)B), dim3(256), sizeof(double) * n, s, mat, n, m, epsilon,
                       gauss, seed, counter, env_base);
    return hipGetLastError();
}

hipError_t launch_filtered_soft_map(const int64_t *picked, const int64_t *topm, int64_t B, int n, int m, int M,
                                    uint64_t seed, uint32_t counter, int64_t env_base, int64_t *out, int *err,
                                    hipStream_t s) {
    const int64_t rows = B * n;
    hipLaunchKernelGGL(filtered_soft_map_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, picked, topm, B,
                       n, m, M, seed, counter, env_base, out, err);
    return hipGetLastError();
}

}  // namespace asg
