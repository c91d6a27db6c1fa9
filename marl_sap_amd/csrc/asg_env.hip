// asg_env.hip -- batched MockConstellationEnv kernels for gfx950.
//
// One workgroup advances one env.  The EpisodeBatch tensors (PyTorch-owned, any
// strides) are written in place: the next pre-transition row (obs, beta, avail_actions,
// prev_assigns, filled) and this step's post-transition row (rewards, terminated,
// actions_onehot).  Benefits come from one of two sources:
//   * BumpSrc  (Philox, native throughput mode): bump parameters are regenerated on the
//     fly from a counter-based key each step -- no benefit table in HBM at all;
//   * ParSrc   (MT19937 compat): the reset's recorded draws [E][m][n] (float64 values) and
//     their float32 table [E][T][n][m] (the rows);
//   * TableSrc (injected): float64 table [E][T][n][m].
// Reference: envs/mock_constellation_env.py:94-175 (reset / step / pre-transition data),
// runners/episode_runner.py:60-100 and runners/parallel_runner.py:113-200 (which rows
// get which fields), components/transforms.py:12-22 (OneHot, int64).
#include "asg_device.h"
#include "asg_internal.h"
#include "lsa_wave.h"

#include <mutex>

namespace asg {

// ------------------------------------------------------------------------------------
// benefit sources.  A source is bound to one env (`bind`) and yields per-pair evaluators.
// ------------------------------------------------------------------------------------
struct BumpSrc {  // Philox, float32 bumps regenerated on the fly (no table in HBM)
    uint64_t seed;
    int64_t env_base;
    uint32_t episode;
    int n, m, T;
    float wmin, wmax;
    bool dense;

    static constexpr bool kNeedsScale = true;
    struct Env {
        EnvKey key;
        uint32_t episode;
        int m, T;
        float wmin, wmax;
        bool dense;
        const float *scale;  // LDS [m]
        struct Pair {
            Bump32 b;
            __device__ float at(int t) const { return bump32_at(b, t); }
            __device__ double at64(int t) const { return bump64_at(b, t); }
        };
        __device__ Pair pair(int i, int j) const {
            return Pair{philox_bump32(key, episode, i * m + j, scale[j], T, wmin, wmax, dense)};
        }
        // pairs (i, j) .. (i, j + 3): one Philox call when they share one (pair index % 4 == 0)
        __device__ void pair4(int i, int j, Pair (&P)[4]) const {
            const int p = i * m + j;
            if ((p & 3) == 0) {
                const float sc[4] = {scale[j], scale[j + 1], scale[j + 2], scale[j + 3]};
                Bump32 b[4];
                philox_bump32x4(key, episode, p, sc, bump_shape(T, wmin, wmax), dense, b);
#pragma unroll
                for (int q = 0; q < 4; ++q) P[q].b = b[q];
                return;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) P[q] = pair(i, j + q);
        }
    };
    // fills scale[0..m) cooperatively (caller syncs)
    __device__ void fill_scale(int64_t e, float *scale) const {
        const EnvKey key = env_key(seed, env_base + e);
        for (int j = threadIdx.x; j < m; j += blockDim.x) scale[j] = philox_task_scale(key, episode, j);
    }
    __device__ Env bind(int64_t e, const float *scale) const {
        return Env{env_key(seed, env_base + e), episode, m, T, wmin, wmax, dense, scale};
    }
};

struct TableSrc {  // float64 table [E][T][n][m] (injected)
    const double *tab;
    int n, m, T;

    static constexpr bool kNeedsScale = false;
    struct Env {
        const double *p;  // &tab[e][0][0][0]
        int m;
        int64_t nm;
        struct Pair {
            const double *p;
            int64_t tstride;
            __device__ double at(int t) const { return p[t * tstride]; }
            __device__ double at64(int t) const { return p[t * tstride]; }
        };
        __device__ Pair pair(int i, int j) const { return Pair{p + (int64_t)i * m + j, nm}; }
        __device__ void pair4(int i, int j, Pair (&P)[4]) const {
#pragma unroll
            for (int q = 0; q < 4; ++q) P[q] = pair(i, j + q);
        }
    };
    __device__ void fill_scale(int64_t, float *) const {}
    __device__ Env bind(int64_t e, const float *) const {
        const int64_t nm = (int64_t)n * m;
        return Env{tab + e * (int64_t)T * nm, m, nm};
    }
};

// MT19937 compat mode: the rows' float32 benefits from the reset's compact float32 table (per
// (env, t) slice only the bump pairs, in (agent, task) order: tmask marks them, toff gives each
// mask word's first compact index -- every other pair is exactly 0), the float64 ones (rewards,
// export) evaluated from the recorded draws par [E][m][n] (mt_par_value, the function the table
// was written with): no float64 table in HBM
struct ParSrc {
    const float *tab32;
    const double2 *par;
    const uint64_t *tmask;
    const int *toff;
    int n, m, T;

    static constexpr bool kNeedsScale = false;
    struct Env {
        const float *p;  // &tab32[e][0][0] (slice 0; slices are n m floats apart)
        const double2 *q;  // &par[e][0][0]
        const uint64_t *mk;  // &tmask[e][0][0]
        const int *of;       // &toff[e][0][0]
        int n, m, W;
        int64_t nm;
        struct Pair {
            const float *p;  // the pair's slice-0 compact value, or nullptr: no bump (0 at every t)
            const double2 *q;
            int64_t tstride;
            __device__ float at(int t) const { return p ? p[t * tstride] : 0.0f; }
            __device__ double at64(int t) const { return mt_par_value(*q, t); }
        };
        __device__ Pair pair(int i, int j) const {
            const int w = j >> 6, b = j & 63;
            const uint64_t mw = mk[(int64_t)i * W + w];
            const float *v = nullptr;
            if ((mw >> b) & 1ull)
                v = p + of[(int64_t)i * W + w] + __popcll(mw & ((1ull << b) - 1ull));
            return Pair{v, q + (int64_t)j * n + i, nm};
        }
        __device__ void pair4(int i, int j, Pair (&P)[4]) const {
#pragma unroll
            for (int k = 0; k < 4; ++k) P[k] = pair(i, j + k);
        }
    };
    __device__ void fill_scale(int64_t, float *) const {}
    __device__ Env bind(int64_t e, const float *) const {
        const int64_t nm = (int64_t)n * m;
        const int W = (m + 63) >> 6;
        return Env{tab32 + e * (int64_t)T * nm, par + e * nm, tmask + e * n * W, toff + e * n * W, n, m, W, nm};
    }
};

// ------------------------------------------------------------------------------------
// pre-transition row writer: obs = [onehot(assign) | B(k) .. B(k+L-1)] (zeros past T),
// beta = B(k) (zeros when k >= T), avail_actions = 1; optionally actions_onehot of the
// post-transition row `ts_onehot`.  VEC consecutive tasks per work item; every store of
// a wave covers whole 128-B lines of one agent's rows.
// ------------------------------------------------------------------------------------
template <int VEC, class EnvB>
__device__ void write_pre_row(const EnvB &src, const asg_batch_view &bv, int64_t e, int ts, int k, int n, int m,
                              int T, int L, const int *s_assign, int ts_onehot) {
    const int groups = m / VEC;
    const int64_t os = bv.obs.stride[3];
    for (int idx = threadIdx.x; idx < n * groups; idx += blockDim.x) {
        const int i = idx / groups;
        const int j0 = (idx - i * groups) * VEC;
        const int a = s_assign ? s_assign[i] : -1;
        float oh[VEC];
        typename EnvB::Pair P[VEC];
#pragma unroll
        for (int q = 0; q < VEC; ++q) oh[q] = (a == j0 + q) ? 1.0f : 0.0f;
        if constexpr (VEC == 4) {
            src.pair4(i, j0, P);
        } else {
#pragma unroll
            for (int q = 0; q < VEC; ++q) P[q] = src.pair(i, j0 + q);
        }
        float *ob = fptr<float>(bv.obs, e, ts, i, j0);
        if (VEC == 4) {
            *reinterpret_cast<float4 *>(ob) = make_float4(oh[0], oh[1], oh[2], oh[3]);
        } else {
            for (int q = 0; q < VEC; ++q) ob[q * os] = oh[q];
        }
        float b0[VEC];
#pragma unroll
        for (int q = 0; q < VEC; ++q) b0[q] = 0.0f;
        for (int l = 0; l < L; ++l) {
            const int t = k + l;
            float val[VEC];
#pragma unroll
            for (int q = 0; q < VEC; ++q) val[q] = (t < T) ? (float)P[q].at(t) : 0.0f;
            if (l == 0) {
#pragma unroll
                for (int q = 0; q < VEC; ++q) b0[q] = val[q];
            }
            float *o = ob + (int64_t)m * (l + 1) * os;
            if (VEC == 4) {
                *reinterpret_cast<float4 *>(o) = make_float4(val[0], val[1], val[2], val[3]);
            } else {
                for (int q = 0; q < VEC; ++q) o[q * os] = val[q];
            }
        }
        if (L == 0 && k < T) {
#pragma unroll
            for (int q = 0; q < VEC; ++q) b0[q] = (float)P[q].at(k);
        }
        if (bv.beta.ptr) {
            float *bp = fptr<float>(bv.beta, e, ts, i, j0);
            if (VEC == 4) {
                *reinterpret_cast<float4 *>(bp) = make_float4(b0[0], b0[1], b0[2], b0[3]);
            } else {
                for (int q = 0; q < VEC; ++q) bp[q * bv.beta.stride[3]] = b0[q];
            }
        }
        if (bv.avail_actions.ptr) {
            uint8_t *ap = fptr<uint8_t>(bv.avail_actions, e, ts, i, j0);
            if (VEC == 4) {
                *reinterpret_cast<uint32_t *>(ap) = 0x01010101u;
            } else {
                for (int q = 0; q < VEC; ++q) ap[q * bv.avail_actions.stride[3]] = 1;
            }
        }
        if (ts_onehot >= 0 && bv.actions_onehot.ptr) {
            int64_t *hp = fptr<int64_t>(bv.actions_onehot, e, ts_onehot, i, j0);
            if (VEC == 4) {
                reinterpret_cast<longlong2 *>(hp)[0] = make_longlong2(a == j0, a == j0 + 1);
                reinterpret_cast<longlong2 *>(hp)[1] = make_longlong2(a == j0 + 2, a == j0 + 3);
            } else {
                for (int q = 0; q < VEC; ++q) hp[q * bv.actions_onehot.stride[3]] = (a == j0 + q);
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// reset: prev_assigns = first n of a random permutation of m; row ts pre-transition data
// ------------------------------------------------------------------------------------
template <int VEC, class Src>
__global__ void __launch_bounds__(256) reset_kernel(Src src, asg_batch_view bv, EnvState st, int ts,
                                                    bool philox_perm) {
    extern __shared__ int s_dyn[];
    const int64_t e = blockIdx.x;
    const int n = st.n, m = st.m;
    int *perm = s_dyn;                                   // [m]
    float *s_scale = reinterpret_cast<float *>(s_dyn + m);  // [m]
    src.fill_scale(e, s_scale);
    if (philox_perm) {
        // Fisher-Yates from the top, Philox-drawn (distribution of choice(m, n, False))
        for (int j = threadIdx.x; j < m; j += blockDim.x) perm[j] = j;
        __syncthreads();
        if (threadIdx.x == 0) {
            const EnvKey key = env_key(st.seed, st.env_base + e);
            for (int i = m - 1; i >= 1; --i) {
                const u32x4 r = philox4x32_10(u32x4{(uint32_t)i, 0u, kCtrPerm, st.episode}, key.k0, key.k1);
                const int jj = (int)(((uint64_t)r.x * (uint64_t)(i + 1)) >> 32);
                const int t = perm[i];
                perm[i] = perm[jj];
                perm[jj] = t;
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += blockDim.x) st.prev[e * n + i] = perm[i];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        if (bv.prev_assigns.ptr)
            *fptr<int64_t>(bv.prev_assigns, e, ts, i, 0) =
                (st.quirks & ASG_QUIRK_PREV_ASSIGNS_ZERO) ? 0 : st.prev[e * n + i];
    }
    if (threadIdx.x == 0) {
        st.returns[e] = 0.0;
        if (bv.filled.ptr) *fptr<int64_t>(bv.filled, e, ts, 0, 0) = 1;
    }
    write_pre_row<VEC>(src.bind(e, s_scale), bv, e, ts, 0, n, m, st.T, st.L, nullptr, -1);
}

// ------------------------------------------------------------------------------------
// bids_as_actions: assignments = LSA(bids, maximize)[1]  (mock :121-122), one wave per
// env, ahead of the step kernel; result in st.assign [E][n]
// ------------------------------------------------------------------------------------
template <int CPL>
__global__ void __launch_bounds__(64) bids_assign_kernel(asg_batch_view bv, EnvState st, int ts) {
    extern __shared__ double s_lsa[];
    const int64_t e = blockIdx.x;
    const int n = st.n, m = st.m;
    float *cost = reinterpret_cast<float *>(s_lsa);  // [n][m] (m > 64)
    const float *bids = fptr<float>(bv.actions, e, ts, 0, 0);
    int c4r[CPL];
    int status;
    if constexpr (CPL == 1) {  // m <= 64: the working matrix stays in registers
        RegCostF32 rc;
        status = lsa_stage_regs<float>(bids, bv.actions.stride[2], bv.actions.stride[3], n, m, true, rc);
        if (status == ASG_OK) status = lsa_solve_reg64(rc, n, m, c4r);
    } else {
        status = lsa_stage_wave<float, float>(bids, bv.actions.stride[2], bv.actions.stride[3], n, m, true, cost);
        if (status == ASG_OK) status = lsa_solve_wave<CPL>(DenseCost<float>{cost, m}, n, m, c4r);
    }
    if (status == ASG_OK) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int i = (int)threadIdx.x + kWave * c;
            if (i < n) st.assign[e * n + i] = c4r[c];
        }
    }
    if (status != ASG_OK) {
        for (int i = threadIdx.x; i < n; i += kWave) st.assign[e * n + i] = -1;
        if (threadIdx.x == 0) atomicCAS(st.err, 0, status);
    }
}

// ------------------------------------------------------------------------------------
// step (mock_constellation_env.py:116-162 plus the runner's batch updates)
// ------------------------------------------------------------------------------------
#ifdef ASG_STEP_WAVES_PER_EU
#define ASG_STEP_VGPR_ATTR __attribute__((amdgpu_waves_per_eu(ASG_STEP_WAVES_PER_EU)))
#else
#define ASG_STEP_VGPR_ATTR
#endif
template <int VEC, class Src, bool BIDS>
__global__ void __launch_bounds__(256) ASG_STEP_VGPR_ATTR step_kernel(Src src, asg_batch_view bv, EnvState st, int ts,
                                                                     int k) {
    extern __shared__ int s_dyn[];
    const int64_t e = blockIdx.x;
    const int n = st.n, m = st.m, T = st.T, L = st.L;
    int *s_act = s_dyn;                                                          // [n]
    int *s_cnt = s_act + n;                                                      // [m]
    float *s_scale = reinterpret_cast<float *>(s_cnt + m);                       // [m]
    double *s_rew = reinterpret_cast<double *>(s_scale + m + ((n + 2 * m) & 1));  // [n], 8-aligned
    __shared__ int s_err;

    if (threadIdx.x == 0) s_err = 0;
    for (int j = threadIdx.x; j < m; j += blockDim.x) s_cnt[j] = 0;
    src.fill_scale(e, s_scale);
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        int a;
        if (BIDS) {
            a = st.assign[e * n + i];
        } else {
            const int64_t a64 = *fptr<int64_t>(bv.actions, e, ts, i, 0);
            a = (a64 >= 0 && a64 < m) ? (int)a64 : -1;
            if (a < 0) s_err = ASG_E_ACTION_RANGE;
        }
        a = a < 0 ? 0 : a;
        s_act[i] = a;
        atomicAdd(&s_cnt[a], 1);
    }
    __syncthreads();
    const auto env = src.bind(e, s_scale);
    // rewards (mock :126-138): only the chosen task's beta_hat is needed per agent
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int j = s_act[i];
        const int p = st.prev[e * n + i];
        const double beta = env.pair(i, j).at64(k);  // float64: mask and reward exact on the parameters
        const double tt = st.T_trans ? st.T_trans[(int64_t)p * m + j] : (j == p ? 0.0 : 1.0);
        const double pen = tt * (beta > 1e-12 ? 1.0 : 0.0);
        const double bh = beta - st.lambda_ * pen;
        const double r = bh > 0.0 ? bh / (double)s_cnt[j] : bh;
        s_rew[i] = r;
        if (bv.rewards.ptr) *fptr<float>(bv.rewards, e, ts, i, 0) = (float)r;
        st.prev[e * n + i] = j;
        if (bv.prev_assigns.ptr)
            *fptr<int64_t>(bv.prev_assigns, e, ts + 1, i, 0) = (st.quirks & ASG_QUIRK_PREV_ASSIGNS_ZERO) ? 0 : j;
    }
    // next pre-transition row (mock :141-160) + this row's OneHot of the actions
    write_pre_row<VEC>(env, bv, e, ts + 1, k + 1, n, m, T, L, s_act, BIDS ? -1 : ts);
    __syncthreads();
    if (threadIdx.x == 0) {
        // episode_return += sum(rewards): Python sums the float64 list left to right
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += s_rew[i];
        st.returns[e] += s;
        bool term = k + 1 >= T;  // terminated = done != info.get("T", False)
        if (st.quirks & ASG_QUIRK_PARALLEL_TERMINATED) term = (e != 0);
        if (bv.terminated.ptr) *fptr<uint8_t>(bv.terminated, e, ts, 0, 0) = term;
        if (bv.filled.ptr) *fptr<int64_t>(bv.filled, e, ts + 1, 0, 0) = 1;
        if (s_err) atomicCAS(st.err, 0, s_err);
    }
}

// ------------------------------------------------------------------------------------
// uniform random actions (BASELINE config 2 random policy)
// ------------------------------------------------------------------------------------
__global__ void random_actions_kernel(asg_batch_view bv, EnvState st, int ts, int k) {
    const int64_t e = blockIdx.x;
    const EnvKey key = env_key(st.seed, st.env_base + e);
    for (int i = threadIdx.x; i < st.n; i += blockDim.x) {
        const u32x4 r = philox4x32_10(u32x4{(uint32_t)i, (uint32_t)k, kCtrAction, st.episode}, key.k0, key.k1);
        *fptr<int64_t>(bv.actions, e, ts, i, 0) = (int64_t)(((uint64_t)r.x * (uint64_t)st.m) >> 32);
    }
}

// ------------------------------------------------------------------------------------
// the random policy's whole episode in one launch (asg_random_rollout): for steps k0 ..
// k0 + steps - 1 of every env, the uniform actions of asg_random_actions (same Philox
// counters) and the transition of step_kernel, optionally after the reset of reset_kernel
// (same Fisher-Yates draws) -- one workgroup per env keeps prev_assigns, the actions, the
// task scales and the return in LDS across the steps; results are those of asg_reset +
// T x (asg_random_actions + asg_step), bit for bit.  Reference: mock_constellation_env.py:
// 94-162 (reset / step) driven by episode_runner.py:60-100 with a uniform policy.
// ------------------------------------------------------------------------------------
template <int VEC, class Src>
__global__ void __launch_bounds__(256) random_rollout_kernel(Src src, asg_batch_view bv, EnvState st, int ts0,
                                                             int k0, int steps, int reset) {
    extern __shared__ int s_dyn[];
    const int64_t e = blockIdx.x;
    const int n = st.n, m = st.m, T = st.T, L = st.L;
    int *s_act = s_dyn;                                                          // [n]
    int *s_cnt = s_act + n;                                                      // [m] (the reset's permutation)
    float *s_scale = reinterpret_cast<float *>(s_cnt + m);                       // [m]
    int *s_prev = reinterpret_cast<int *>(s_scale + m);                          // [n]
    double *s_rew = reinterpret_cast<double *>(s_prev + n + ((2 * n + 2 * m) & 1));  // [n], 8-aligned
    __shared__ double s_ret;
    src.fill_scale(e, s_scale);
    const auto env = src.bind(e, s_scale);
    const EnvKey key = env_key(st.seed, st.env_base + e);
    if (reset) {
        // reset_kernel: Fisher-Yates from the top, Philox-drawn, one thread (the same draws)
        for (int j = threadIdx.x; j < m; j += blockDim.x) s_cnt[j] = j;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int i = m - 1; i >= 1; --i) {
                const u32x4 r = philox4x32_10(u32x4{(uint32_t)i, 0u, kCtrPerm, st.episode}, key.k0, key.k1);
                const int jj = (int)(((uint64_t)r.x * (uint64_t)(i + 1)) >> 32);
                const int t = s_cnt[i];
                s_cnt[i] = s_cnt[jj];
                s_cnt[jj] = t;
            }
            s_ret = 0.0;
            if (bv.filled.ptr) *fptr<int64_t>(bv.filled, e, ts0, 0, 0) = 1;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            s_prev[i] = s_cnt[i];
            if (bv.prev_assigns.ptr)
                *fptr<int64_t>(bv.prev_assigns, e, ts0, i, 0) = (st.quirks & ASG_QUIRK_PREV_ASSIGNS_ZERO) ? 0 : s_cnt[i];
        }
        write_pre_row<VEC>(env, bv, e, ts0, 0, n, m, T, L, nullptr, -1);
    } else {
        for (int i = threadIdx.x; i < n; i += blockDim.x) s_prev[i] = st.prev[e * n + i];
        if (threadIdx.x == 0) s_ret = st.returns[e];
    }
    for (int it = 0; it < steps; ++it) {
        const int k = k0 + it, ts = ts0 + it;
        __syncthreads();  // the previous step's counts / actions are consumed
        for (int j = threadIdx.x; j < m; j += blockDim.x) s_cnt[j] = 0;
        __syncthreads();
        // random_actions_kernel's draw: action of agent i at step k
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const u32x4 r = philox4x32_10(u32x4{(uint32_t)i, (uint32_t)k, kCtrAction, st.episode}, key.k0, key.k1);
            const int a = (int)(((uint64_t)r.x * (uint64_t)m) >> 32);
            if (bv.actions.ptr) *fptr<int64_t>(bv.actions, e, ts, i, 0) = a;
            s_act[i] = a;
            atomicAdd(&s_cnt[a], 1);
        }
        __syncthreads();
        // step_kernel's rewards (mock :126-138)
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const int j = s_act[i];
            const int p = s_prev[i];
            const double beta = env.pair(i, j).at64(k);
            const double tt = st.T_trans ? st.T_trans[(int64_t)p * m + j] : (j == p ? 0.0 : 1.0);
            const double pen = tt * (beta > 1e-12 ? 1.0 : 0.0);
            const double bh = beta - st.lambda_ * pen;
            const double r = bh > 0.0 ? bh / (double)s_cnt[j] : bh;
            s_rew[i] = r;
            if (bv.rewards.ptr) *fptr<float>(bv.rewards, e, ts, i, 0) = (float)r;
            s_prev[i] = j;
            if (bv.prev_assigns.ptr)
                *fptr<int64_t>(bv.prev_assigns, e, ts + 1, i, 0) = (st.quirks & ASG_QUIRK_PREV_ASSIGNS_ZERO) ? 0 : j;
        }
        write_pre_row<VEC>(env, bv, e, ts + 1, k + 1, n, m, T, L, s_act, ts);
        __syncthreads();
        if (threadIdx.x == 0) {
            double sum = 0.0;  // Python's sum(rewards), left to right
            for (int i = 0; i < n; ++i) sum += s_rew[i];
            s_ret += sum;
            bool term = k + 1 >= T;
            if (st.quirks & ASG_QUIRK_PARALLEL_TERMINATED) term = (e != 0);
            if (bv.terminated.ptr) *fptr<uint8_t>(bv.terminated, e, ts, 0, 0) = term;
            if (bv.filled.ptr) *fptr<int64_t>(bv.filled, e, ts + 1, 0, 0) = 1;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) st.prev[e * n + i] = s_prev[i];
    if (threadIdx.x == 0) st.returns[e] = s_ret;
}

// ------------------------------------------------------------------------------------
// table export (Philox bumps -> [E][n][m][T] float64, the reference layout)
// ------------------------------------------------------------------------------------
template <class Src>
__global__ void export_table_kernel(Src src, EnvState st, double *out) {
    extern __shared__ int s_dyn[];
    float *s_scale = reinterpret_cast<float *>(s_dyn);
    const int64_t e = blockIdx.x;
    const int n = st.n, m = st.m, T = st.T;
    src.fill_scale(e, s_scale);
    __syncthreads();
    const auto env = src.bind(e, s_scale);
    for (int p = threadIdx.x; p < n * m; p += blockDim.x) {
        const int i = p / m, j = p - i * m;
        const auto P = env.pair(i, j);
        for (int t = 0; t < T; ++t) out[((e * n + i) * (int64_t)m + j) * T + t] = P.at64(t);
    }
}

// Philox bump parameters [E][n][m][3] float32 = (scale (0: inactive pair), center, a2), the
// values every bump evaluation uses (value(t) = scale * 2^(-(t - center)^2 * a2))
__global__ void export_bump_params_kernel(BumpSrc src, EnvState st, float *out) {
    extern __shared__ int s_dyn[];
    float *s_scale = reinterpret_cast<float *>(s_dyn);
    const int64_t e = blockIdx.x;
    const int n = st.n, m = st.m;
    src.fill_scale(e, s_scale);
    __syncthreads();
    const auto env = src.bind(e, s_scale);
    for (int p = threadIdx.x; p < n * m; p += blockDim.x) {
        const Bump32 b = env.pair(p / m, p % m).b;
        float *o = out + (e * n * (int64_t)m + p) * 3;
        o[0] = b.scale;
        o[1] = b.center;
        o[2] = b.a2;
    }
}

// [E][n][m][T] (reference layout) -> [E][T][n][m] (kernel layout)
__global__ void import_table_kernel(const double *in, EnvState st, double *tab, int64_t src_envs) {
    const int64_t e = blockIdx.x;
    const int n = st.n, m = st.m, T = st.T;
    const int64_t se = src_envs == 1 ? 0 : e;
    for (int64_t p = threadIdx.x; p < (int64_t)n * m * T; p += blockDim.x) {
        const int t = (int)(p % T);
        const int64_t ij = p / T;
        const double x = in[se * (int64_t)n * m * T + p];
        tab[(e * T + t) * (int64_t)n * m + ij] = x;
        st.table32[(e * T + t) * (int64_t)n * m + ij] = (float)x;
    }
}

__global__ void export_prev_kernel(EnvState st, int64_t *out) {
    const int64_t e = blockIdx.x;
    for (int i = threadIdx.x; i < st.n; i += blockDim.x) out[e * st.n + i] = st.prev[e * st.n + i];
}

// ------------------------------------------------------------------------------------
// legacy MT19937 compat mode: one wave per env, stream state [E][625] in HBM
// ------------------------------------------------------------------------------------
constexpr int kMtN = 624, kMtM = 397;

__global__ void mt_seed_kernel(uint32_t *mt, int64_t E, uint64_t seed, int64_t base, bool replicate) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    uint32_t *key = mt + e * (kMtN + 1);
    uint32_t s = (uint32_t)(replicate ? seed : seed + (uint64_t)(base + e));
    key[0] = s;
    for (int i = 1; i < kMtN; ++i) {
        s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i;
        key[i] = s;
    }
    key[kMtN] = kMtN;  // pos
}

// A wave-cooperative view of one MT19937 stream in LDS with pre-tempered output words.
struct MtWave {
    uint32_t *key;  // [624] raw state (LDS)
    uint32_t *out;  // [624] tempered words (LDS)
    int pos;        // wave-uniform

    __device__ void twist() {
        const int lane = threadIdx.x & (kWave - 1);
        // scipy-free restatement of the MT recurrence in 4 dependency phases
        auto gen = [&](int i, uint32_t ki, uint32_t ki1, uint32_t kim) {
            const uint32_t y = (ki & 0x80000000u) | (ki1 & 0x7fffffffu);
            return kim ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        };
        const int phase_lo[3] = {0, kMtN - kMtM, 2 * (kMtN - kMtM)};
        const int phase_hi[3] = {kMtN - kMtM, 2 * (kMtN - kMtM), kMtN - 1};
        for (int ph = 0; ph < 3; ++ph) {
            uint32_t nv[4];
            int cnt = 0;
            for (int i = phase_lo[ph] + lane; i < phase_hi[ph]; i += kWave, ++cnt)
                nv[cnt] = gen(i, key[i], key[i + 1], key[(i + kMtM) % kMtN]);
            wave_sync();
            cnt = 0;
            for (int i = phase_lo[ph] + lane; i < phase_hi[ph]; i += kWave, ++cnt) key[i] = nv[cnt];
            wave_sync();
        }
        if (lane == 0) key[kMtN - 1] = gen(kMtN - 1, key[kMtN - 1], key[0], key[kMtM - 1]);
        wave_sync();
        temper_all();
        pos = 0;
    }
    __device__ void temper_all() {
        const int lane = threadIdx.x & (kWave - 1);
        for (int i = lane; i < kMtN; i += kWave) {
            uint32_t y = key[i];
            y ^= (y >> 11);
            y ^= (y << 7) & 0x9d2c5680u;
            y ^= (y << 15) & 0xefc60000u;
            y ^= (y >> 18);
            out[i] = y;
        }
        wave_sync();
    }
    __device__ uint32_t next() {
        if (pos >= kMtN) twist();
        return out[pos++];
    }
    __device__ double next_double() {
        const uint32_t a = next() >> 5, b = next() >> 6;
        return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
    }
    __device__ double uniform(double lo, double hi) { return lo + (hi - lo) * next_double(); }
    __device__ uint32_t interval(uint32_t max) {
        if (max == 0) return 0;
        uint32_t mask = max;
        mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
        uint32_t v;
        while ((v = (next() & mask)) > max) {}
        return v;
    }
};

// MT19937 over two LDS blocks: `out` holds the tempered words of the current block (numpy's
// state `key`, position `pos`) and of the next one (`key2`, twisted ahead), so any word up to
// 624 ahead of pos is readable without a twist in between -- what the speculative reads of
// mt_reset_kernel need.  The state handed back is (key, pos): numpy's.
__device__ __forceinline__ void mt_twist_inplace(uint32_t *k) {
    const int lane = threadIdx.x & (kWave - 1);
    auto gen = [&](uint32_t ki, uint32_t ki1, uint32_t kim) {
        const uint32_t y = (ki & 0x80000000u) | (ki1 & 0x7fffffffu);
        return kim ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    };
    const int phase_lo[3] = {0, kMtN - kMtM, 2 * (kMtN - kMtM)};
    const int phase_hi[3] = {kMtN - kMtM, 2 * (kMtN - kMtM), kMtN - 1};
    for (int ph = 0; ph < 3; ++ph) {
        uint32_t nv[4];
        int cnt = 0;
        for (int i = phase_lo[ph] + lane; i < phase_hi[ph]; i += kWave, ++cnt)
            nv[cnt] = gen(k[i], k[i + 1], k[(i + kMtM) % kMtN]);
        wave_sync();
        cnt = 0;
        for (int i = phase_lo[ph] + lane; i < phase_hi[ph]; i += kWave, ++cnt) k[i] = nv[cnt];
        wave_sync();
    }
    if (lane == 0) k[kMtN - 1] = gen(k[kMtN - 1], k[0], k[kMtM - 1]);
    wave_sync();
}
__device__ __forceinline__ void mt_temper(const uint32_t *k, uint32_t *o) {
    const int lane = threadIdx.x & (kWave - 1);
    for (int i = lane; i < kMtN; i += kWave) {
        uint32_t y = k[i];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        o[i] = y;
    }
    wave_sync();
}
// ASG_MT_TEMPER_ON_READ=1: the tempered copies are not kept -- a word is tempered when read (4
// shift / mask steps) -- so a draw wave holds only the two raw blocks, 5 KiB of LDS instead of
// 10 (29 draw waves per CU instead of 16).  Measured slower (r5 A/B, compat leg): 0.946-0.954 vs
// 0.892-0.900 ms/step -- the speculative reads temper every word they test; off
// Timing-only switch (WRONG results; refused without -DASG_TIMING_EXPERIMENTS): ASG_MT_XSKIP bits
// 1 = no twist of the next block at a shift (the tempered words go stale), 2 = no speculative
// bump loop (each task's agents consumed as if none had a bump), 4 = no permutation
#if defined(ASG_MT_XSKIP) && !defined(ASG_TIMING_EXPERIMENTS)
#error "ASG_MT_XSKIP gives wrong results: timing experiments only (-DASG_TIMING_EXPERIMENTS)"
#endif
#ifndef ASG_MT_XSKIP
#define ASG_MT_XSKIP 0
#endif
#ifndef ASG_MT_TEMPER_ON_READ
#define ASG_MT_TEMPER_ON_READ 0
#endif
__device__ __forceinline__ uint32_t mt_temper1(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}
struct MtWave2 {
    uint32_t *key, *key2;  // [624] raw states of the current and the next block (LDS)
    uint32_t *out;         // [1248] tempered words of both (unused with ASG_MT_TEMPER_ON_READ)
    int pos;               // wave-uniform, < 624 between calls
    __device__ void init(int pos0) {
        const int lane = threadIdx.x & (kWave - 1);
        if (!ASG_MT_TEMPER_ON_READ) mt_temper(key, out);
        for (int i = lane; i < kMtN; i += kWave) key2[i] = key[i];
        wave_sync();
        mt_twist_inplace(key2);
        if (!ASG_MT_TEMPER_ON_READ) mt_temper(key2, out + kMtN);
        pos = pos0;
        if (pos >= kMtN) shift();
    }
    __device__ void shift() {  // the next block becomes the current one
        const int lane = threadIdx.x & (kWave - 1);
        for (int i = lane; i < kMtN; i += kWave) {
            key[i] = key2[i];
            if (!ASG_MT_TEMPER_ON_READ) out[i] = out[kMtN + i];
        }
        wave_sync();
        if (!(ASG_MT_XSKIP & 1)) {
            mt_twist_inplace(key2);
            if (!ASG_MT_TEMPER_ON_READ) mt_temper(key2, out + kMtN);
        }
        pos -= kMtN;
    }
    __device__ uint32_t word(int k) const {  // k < 624 (per lane: the speculative reads)
        if (ASG_MT_TEMPER_ON_READ) {
            const int i = pos + k;
            return mt_temper1(i < kMtN ? key[i] : key2[i - kMtN]);
        }
        return out[pos + k];
    }
    __device__ void advance(int c) {
        pos += c;
        if (pos >= kMtN) shift();
    }
    __device__ uint32_t next() {
        const uint32_t w = word(0);
        advance(1);
        return w;
    }
    __device__ static double dbl(uint32_t a, uint32_t b) {  // numpy's random_sample from two words
        return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
    }
    __device__ double next_double() {
        const double d = dbl(word(0), word(1));
        advance(2);
        return d;
    }
    __device__ double uniform(double lo, double hi) { return lo + (hi - lo) * next_double(); }
    __device__ uint32_t interval(uint32_t max) {
        if (max == 0) return 0;
        uint32_t mask = max;
        mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
        uint32_t v;
        while ((v = (next() & mask)) > max) {}
        return v;
    }
};

// generate_benefits_over_time + permutation in MT compat mode, the draws half: one wave per
// env consumes its MT19937 stream in the reference's order (mock :276-299, :105) and records
// each (agent, task) bump of the reset's table -- center and spread, the scale as the sign of spread,
// (0, 0) for no bump -- in par [E][m][n] (draw order: one coalesced 1 KiB store per 64 agents
// of a task); mt_table_kernel then writes the table from them with whole-row stores.
// construct: also replay the throwaway __init__ table draw (mock :34) first.
// bumps resolved per LDS round trip of the draw loop's bump search
#ifndef ASG_MT_BUMPS
#define ASG_MT_BUMPS 8
#endif
constexpr int kMtBumps = ASG_MT_BUMPS;
// numpy's random_sample() from words (a, b) is ((a >> 5) 2^26 + (b >> 6)) 2^-53 exactly: r > 0.75
// (mock :283) is an integer test on the 53-bit numerator against 3 2^51
__device__ __forceinline__ bool mt_r_above_075(uint32_t a, uint32_t b) {
    const uint32_t hi = a >> 5, lo = b >> 6;
    return hi > (3u << 25) || (hi == (3u << 25) && lo != 0u);
}
__global__ void __launch_bounds__(64) mt_reset_kernel(uint32_t *mtstate, EnvState st, double2 *par, bool construct,
                                                       bool generate, int64_t e0 = 0) {
    extern __shared__ uint32_t s_mt[];
    uint32_t *key = s_mt, *key2 = s_mt + kMtN, *out = s_mt + 2 * kMtN;
    int *perm = reinterpret_cast<int *>(out + (ASG_MT_TEMPER_ON_READ ? 0 : 2 * kMtN));
    const int64_t e = e0 + blockIdx.x;
    const int lane = threadIdx.x;
    const int n = st.n, m = st.m, T = st.T;
    uint32_t *g = mtstate + e * (kMtN + 1);
    for (int i = lane; i < kMtN; i += kWave) key[i] = g[i];
    wave_sync();
    MtWave2 mt{key, key2, out, 0};
    mt.init((int)g[kMtN]);
    double2 *pe = par ? par + e * (int64_t)n * m : nullptr;
    for (int pass = construct ? 0 : 1; generate && pass < 2; ++pass) {
        const double wmin = pass == 0 ? st.wmin_init : st.wmin;
        const double wmax = pass == 0 ? st.wmax_init : st.wmax;
        for (int j = 0; j < m; ++j) {
            // benefit_scale = choice([1, 1, 1, 10]): one word (randint(0, 4), mask 3), read with the
            // first chunk's words (the chunk's offsets start after it: o0)
            const double scale = (mt.word(0) & 3u) == 3u ? 10.0 : 1.0;
            int o0 = 1;
            for (int c0 = 0; c0 < n; c0 += kWave) {
                const int rows = min(n, c0 + kWave) - c0;
                // 1. which agents of the chunk have a bump (r > 0.75): lane l tests agent a0 + l with
                //    its two r words at o + 2 l + 4 s, s = the bumps before it among a0.., s <
                //    kMtBumps -- all read in one LDS round trip, the first hit at s = 0 is exact, the
                //    first after it at s = 1, ... (integer tests, no float64); no stream advance yet
                uint64_t bumps = 0;
                int o = o0, a0 = 0;  // o0 + the words consumed by agents 0 .. a0 - 1 of the chunk
                if (ASG_MT_XSKIP & 2) a0 = rows;
                while (a0 < rows) {
                    uint32_t rw[2 * kMtBumps];
#pragma unroll
                    for (int q = 0; q < 2 * kMtBumps; ++q) rw[q] = mt.word(o + 2 * lane + 4 * (q >> 1) + (q & 1));
                    int lo = 0, found = 0;
                    bool done = false;
#pragma unroll
                    for (int sb = 0; sb < kMtBumps; ++sb) {
                        const uint64_t act = __ballot(lane + a0 < rows && lane >= lo && mt_r_above_075(rw[2 * sb], rw[2 * sb + 1]));
                        if (act == 0) {
                            done = true;
                            break;
                        }
                        const int k = __builtin_amdgcn_readfirstlane(__builtin_ctzll(act));
                        bumps |= 1ull << (a0 + k);
                        lo = k + 1;
                        found = sb + 1;
                    }
                    if (done) {  // agents a0 .. rows - 1: two words each, four more per bump
                        o += 2 * (rows - a0) + 4 * found;
                        a0 = rows;
                    } else {
                        o += 2 * lo + 4 * found;
                        a0 += lo;
                    }
                }
                // 2. every bump's center and spread read by its own lane: agent l's words start at
                //    o0 + 2 l + 4 (bumps before l); center ~ U(0, T), spread ~ U(wmin, wmax) (numpy's
                //    uniform(lo, hi) = lo + (hi - lo) * random_sample(), as MtWave2::uniform)
                double2 mine = make_double2(0.0, 0.0);  // agent c0 + lane's bump on task j
                if ((bumps >> lane) & 1) {
                    const int sl = __builtin_amdgcn_mbcnt_hi((uint32_t)(bumps >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)bumps, 0u));
                    const int w = o0 + 2 * lane + 4 * sl + 2;
                    const double center = 0.0 + ((double)T - 0.0) * MtWave2::dbl(mt.word(w), mt.word(w + 1));
                    const double spread = wmin + (wmax - wmin) * MtWave2::dbl(mt.word(w + 2), mt.word(w + 3));
                    mine = make_double2(center, scale == 10.0 ? -spread : spread);  // s2 in mt_table_kernel
                }
                mt.advance(o);
                o0 = 0;
                if (pass == 1 && pe && c0 + lane < n) pe[(int64_t)j * n + c0 + lane] = mine;
            }
        }
    }
    // prev_assigns = choice(m, n, replace=False) = permutation(m)[:n]  (mock :105)
    for (int j = lane; j < m; j += kWave) perm[j] = j;
    wave_sync();
    for (int i = (ASG_MT_XSKIP & 4) ? 0 : m - 1; i >= 1; --i) {
        const int jj = (int)mt.interval((uint32_t)i);
        if (lane == 0) {
            const int t = perm[i];
            perm[i] = perm[jj];
            perm[jj] = t;
        }
        wave_sync();
    }
    for (int i = lane; i < n; i += kWave) st.prev[e * n + i] = perm[i];
    for (int i = lane; i < kMtN; i += kWave) g[i] = key[i];
    if (lane == 0) g[kMtN] = (uint32_t)mt.pos;
}

// the reset's table B[e][t][i][j] = mt_par_value(draw, t) (the reference's zeros + bumps, mock
// :276-299) rounded to float32, the rows' dtype, stored COMPACT: per (env, t) slice only the
// bump pairs (about one in four; every other value is exactly 0), in (agent, task) order, with
// their masks tmask [E][n][W] and each mask word's first compact index toff [E][n][W] -- the
// episode kernel then reads ~1/4 of a dense slice per lookahead block.  Per chunk of `rows`
// agents (rows * m <= 1024): the draws staged transposed in LDS, the chunk's pair masks built
// (LDS 64-bit OR) and the compact order listed; then one thread per bump evaluates its T values
// (the float64 sigma_2 once, the exp / division per value: for bumps only) and stores them
// straight into the T slices -- consecutive threads, consecutive compact indices.  The float64
// values are not stored: their readers evaluate them from the draws (ParSrc).
#ifndef ASG_TABLE_ROWS
#define ASG_TABLE_ROWS 16
#endif
static int mt_table_rows(int m) {
    return m >= 1024 ? 1 : (1024 / m < ASG_TABLE_ROWS ? 1024 / m : ASG_TABLE_ROWS);
}
static size_t mt_table_lds(int R, int m) {
    const size_t W = (m + 63) / 64;
    return (sizeof(double2) + sizeof(int)) * (size_t)R * m + 8 + (sizeof(uint64_t) + sizeof(int)) * (size_t)R * W;
}
__global__ void __launch_bounds__(256) mt_table_kernel(const double2 *par, EnvState st, int R, int64_t e0 = 0) {
    extern __shared__ double2 s_par[];                               // [R agents][m tasks]
    int *s_list = reinterpret_cast<int *>(s_par + R * st.m);         // the chunk's bumps, compact order
    const int W = (st.m + 63) >> 6;
    unsigned long long *s_mask = reinterpret_cast<unsigned long long *>(s_list + R * st.m + ((R * st.m) & 1));
    int *s_off = reinterpret_cast<int *>(s_mask + R * W);           // [R][W] compact index (chunk-relative)
    __shared__ int s_cnt;
    const int64_t e = e0 + blockIdx.x;
    const int n = st.n, m = st.m, T = st.T;
    const int64_t nm = (int64_t)n * m;
    const double2 *pe = par + e * nm;
    float *te = st.table32 + e * T * nm;
    uint64_t *gm = st.tmask + e * n * W;
    int *go = st.toff + e * n * W;
    int base = 0;  // the env's compact index of the chunk's first bump
    for (int i0 = 0; i0 < n; i0 += R) {
        const int rows = min(R, n - i0), ne = rows * m;
        __syncthreads();
        // par is [task][agent]: `rows` consecutive agents of a task are contiguous
        for (int idx = threadIdx.x; idx < ne; idx += blockDim.x) {
            const int ii = idx % rows, j = idx / rows;
            s_par[ii * m + j] = pe[(int64_t)j * n + i0 + ii];
        }
        for (int x = threadIdx.x; x < rows * W; x += blockDim.x) s_mask[x] = 0ull;
        __syncthreads();
        for (int idx = threadIdx.x; idx < ne; idx += blockDim.x)
            if (s_par[idx].y != 0.0) {
                const int ii = idx / m, j = idx - ii * m;
                atomicOr(&s_mask[ii * W + (j >> 6)], 1ull << (j & 63));
            }
        __syncthreads();
        if (threadIdx.x == 0) {  // exclusive prefix over the chunk's mask words, (agent, word) order
            int c = 0;
            for (int x = 0; x < rows * W; ++x) {
                s_off[x] = c;
                c += __popcll(s_mask[x]);
            }
            s_cnt = c;
        }
        __syncthreads();
        for (int x = threadIdx.x; x < rows * W; x += blockDim.x) {
            gm[(int64_t)i0 * W + x] = s_mask[x];
            go[(int64_t)i0 * W + x] = base + s_off[x];
        }
        // each bump's slot in the compact order
        for (int idx = threadIdx.x; idx < ne; idx += blockDim.x)
            if (s_par[idx].y != 0.0) {
                const int ii = idx / m, j = idx - ii * m, w = ii * W + (j >> 6);
                s_list[s_off[w] + __popcll(s_mask[w] & ((1ull << (j & 63)) - 1ull))] = idx;
            }
        __syncthreads();
        const int cnt = s_cnt;
        float *o = te + base;
        for (int k = threadIdx.x; k < cnt; k += blockDim.x) {
            const double2 p = s_par[s_list[k]];
            // mt_par_value(p, t) for every t, sigma_2 hoisted (the same float64 operations)
            const double scale = p.y < 0.0 ? 10.0 : 1.0, s2 = bump_s2(__builtin_fabs(p.y));
            for (int t = 0; t < T; ++t) o[(int64_t)t * nm + k] = (float)bump_value(scale, p.x, s2, t);
        }
        base += cnt;
    }
}

// skip `words` draws of every stream (other consumers of numpy's global stream)
__global__ void __launch_bounds__(64) mt_advance_kernel(uint32_t *mtstate, int64_t words) {
    extern __shared__ uint32_t s_mt[];
    uint32_t *key = s_mt, *out = s_mt + kMtN;
    const int64_t e = blockIdx.x;
    uint32_t *g = mtstate + e * (kMtN + 1);
    for (int i = threadIdx.x; i < kMtN; i += kWave) key[i] = g[i];
    wave_sync();
    MtWave mt{key, out, (int)g[kMtN]};
    int64_t left = words;
    while (left > 0) {
        if (mt.pos >= kMtN) mt.twist();
        const int64_t take = min<int64_t>(left, kMtN - mt.pos);
        mt.pos += (int)take;
        left -= take;
    }
    for (int i = threadIdx.x; i < kMtN; i += kWave) g[i] = key[i];
    if (threadIdx.x == 0) g[kMtN] = (uint32_t)mt.pos;
}

// ------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------
// float4 / uchar4 / 2x longlong2 row stores need unit inner stride, 4-element aligned
// outer strides and aligned base pointers
static bool vec4_ok(const asg_batch_view &b, int m) {
    auto al = [](const asg_field &f, uintptr_t bytes) {
        if (!f.ptr) return true;
        if (f.stride[3] != 1 || reinterpret_cast<uintptr_t>(f.ptr) % bytes) return false;
        return f.stride[0] % 4 == 0 && f.stride[1] % 4 == 0 && f.stride[2] % 4 == 0;
    };
    return m % 4 == 0 && al(b.obs, 16) && al(b.beta, 16) && al(b.avail_actions, 4) &&
           al(b.actions_onehot, 16);
}

static size_t step_lds_bytes(const EnvState &st) {
    return sizeof(int) * (st.n + 2 * st.m + 1) + sizeof(double) * st.n + 16;
}

template <class Src, bool BIDS>
static void launch_step_t(const Src &src, const asg_batch_view &bv, const EnvState &st, int ts, int k,
                          hipStream_t s) {
    const size_t lds = step_lds_bytes(st);
    if (vec4_ok(bv, st.m))
        hipLaunchKernelGGL((step_kernel<4, Src, BIDS>), dim3(st.E), dim3(256), lds, s, src, bv, st, ts, k);
    else
        hipLaunchKernelGGL((step_kernel<1, Src, BIDS>), dim3(st.E), dim3(256), lds, s, src, bv, st, ts, k);
}

hipError_t launch_bids_assign(const asg_batch_view &bv, const EnvState &st, int ts, hipStream_t s) {
    const size_t lds = sizeof(float) * (size_t)st.n * st.m + 32;
    // bids matrices are at most 16384 entries (checked at create): m <= 16384 / n
    if (st.m <= 64) hipLaunchKernelGGL(bids_assign_kernel<1>, dim3(st.E), dim3(64), lds, s, bv, st, ts);
    else if (st.m <= 128) hipLaunchKernelGGL(bids_assign_kernel<2>, dim3(st.E), dim3(64), lds, s, bv, st, ts);
    else if (st.m <= 256) hipLaunchKernelGGL(bids_assign_kernel<4>, dim3(st.E), dim3(64), lds, s, bv, st, ts);
    else if (st.m <= 512) hipLaunchKernelGGL(bids_assign_kernel<8>, dim3(st.E), dim3(64), lds, s, bv, st, ts);
    else hipLaunchKernelGGL(bids_assign_kernel<16>, dim3(st.E), dim3(64), lds, s, bv, st, ts);
    return hipGetLastError();
}

template <class Src>
static hipError_t launch_step_src(const Src &src, const asg_batch_view &bv, const EnvState &st, int ts, int k,
                                  hipStream_t s, bool assign_ready) {
    if (st.bids) {
        if (!assign_ready) {
            const hipError_t e = launch_bids_assign(bv, st, ts, s);
            if (e != hipSuccess) return e;
        }
        launch_step_t<Src, true>(src, bv, st, ts, k, s);
    } else {
        launch_step_t<Src, false>(src, bv, st, ts, k, s);
    }
    return hipGetLastError();
}

template <class Src>
static hipError_t launch_reset_src(const Src &src, const asg_batch_view &bv, const EnvState &st, int ts,
                                   bool philox_perm, hipStream_t s) {
    const size_t lds = sizeof(int) * 2 * st.m + 16;
    if (vec4_ok(bv, st.m))
        hipLaunchKernelGGL((reset_kernel<4, Src>), dim3(st.E), dim3(256), lds, s, src, bv, st, ts, philox_perm);
    else
        hipLaunchKernelGGL((reset_kernel<1, Src>), dim3(st.E), dim3(256), lds, s, src, bv, st, ts, philox_perm);
    return hipGetLastError();
}

static BumpSrc bump_src(const EnvState &st) {
    return BumpSrc{st.seed, st.env_base, st.episode, st.n, st.m, st.T, (float)st.wmin, (float)st.wmax,
                   st.benefit_mode == ASG_BENEFIT_DENSE};
}
static TableSrc table_src(const EnvState &st) { return TableSrc{st.table, st.n, st.m, st.T}; }
static ParSrc par_src(const EnvState &st) { return ParSrc{st.table32, st.mtpar, st.tmask, st.toff, st.n, st.m, st.T}; }

static bool uses_table(const EnvState &st) {
    return st.rng_mode == ASG_RNG_MT19937 || st.benefit_mode == ASG_BENEFIT_INJECTED;
}

hipError_t launch_reset(const asg_batch_view &bv, const EnvState &st, int ts, bool construct, hipStream_t s) {
    if (st.rng_mode == ASG_RNG_MT19937) {
        // the two raw MT19937 blocks + the permutation: 5,248 B at m = 64 (29 workgroups in a
        // CU's 160 KiB, LDS in 512-byte granules); with the tempered copies kept
        // (ASG_MT_TEMPER_ON_READ=0) 10,240 B, exactly 16 workgroups
        // with an injected table (sat_prox_mat=) neither __init__ nor reset draw a
        // table: only the permutation consumes the stream (mock :32-37, :99-105)
        const bool gen = st.benefit_mode != ASG_BENEFIT_INJECTED;
        hipError_t err = launch_reset_draws(st, construct, s);
        if (err != hipSuccess) return err;
        return gen ? launch_reset_src(par_src(st), bv, st, ts, false, s)
                   : launch_reset_src(table_src(st), bv, st, ts, false, s);
    }
    if (uses_table(st)) return launch_reset_src(table_src(st), bv, st, ts, true, s);
    return launch_reset_src(bump_src(st), bv, st, ts, true, s);
}

// The MT19937 mode's reset without its row write: the draws (and the float32 table) only --
// the episode launch that follows writes the reset row (asg_reset_rollout in the same-seed mode)
// The draws (one wave per env, latency-bound: the sequential MT19937 consumption) and the table
// writer (float64 bump evaluations, compute-bound) are pipelined over env chunks on two streams:
// chunk c's table kernel runs on an auxiliary stream beside chunk c + 1's draws (disjoint envs),
// each table chunk after its own draws (an event) and after everything before the reset on the
// caller's stream (so the previous episode's table readers are done), the caller's stream waiting
// for the last table chunk.  One auxiliary stream and event set per device (handles of one device
// used from several host threads at once would share them).
#ifndef ASG_RESET_CHUNKS
#define ASG_RESET_CHUNKS 1  // 2 / 4 / 8 measured no faster (r6 A/B): one launch each
#endif
namespace {
struct ResetAux {
    hipStream_t s = nullptr;
    hipEvent_t ev[ASG_RESET_CHUNKS + 1] = {};
};
hipError_t reset_aux(ResetAux **out) {
    static std::mutex mu;
    static ResetAux aux[64];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(mu);
    ResetAux &a = aux[dev];
    if (!a.s) {
        if ((e = hipStreamCreateWithFlags(&a.s, hipStreamNonBlocking)) != hipSuccess) return e;
        for (auto &ev : a.ev)
            if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
    }
    *out = &a;
    return hipSuccess;
}
}  // namespace

hipError_t launch_reset_draws(const EnvState &st, bool construct, hipStream_t s) {
    if (st.rng_mode != ASG_RNG_MT19937) return hipErrorInvalidValue;
    const size_t lds = sizeof(uint32_t) * (ASG_MT_TEMPER_ON_READ ? 2 : 4) * kMtN + sizeof(int) * st.m;
    const bool gen = st.benefit_mode != ASG_BENEFIT_INJECTED;
    const int R = mt_table_rows(st.m);
    const int K = (gen && st.E >= 1024) ? ASG_RESET_CHUNKS : 1;
    if (K == 1) {
        hipLaunchKernelGGL(mt_reset_kernel, dim3(st.E), dim3(64), lds, s, st.mt, st, st.mtpar, construct && gen, gen,
                           (int64_t)0);
        hipError_t err = hipGetLastError();
        if (err != hipSuccess || !gen) return err;
        hipLaunchKernelGGL(mt_table_kernel, dim3(st.E), dim3(256), mt_table_lds(R, st.m), s, st.mtpar, st, R,
                           (int64_t)0);
        return hipGetLastError();
    }
    ResetAux *ax = nullptr;
    hipError_t err = reset_aux(&ax);
    if (err != hipSuccess) return err;
    for (int c = 0; c < K; ++c) {
        const int64_t e0 = st.E * c / K, e1 = st.E * (c + 1) / K;
        hipLaunchKernelGGL(mt_reset_kernel, dim3((unsigned)(e1 - e0)), dim3(64), lds, s, st.mt, st, st.mtpar,
                           construct, true, e0);
        if ((err = hipGetLastError()) != hipSuccess) return err;
        if ((err = hipEventRecord(ax->ev[c], s)) != hipSuccess) return err;
        if ((err = hipStreamWaitEvent(ax->s, ax->ev[c], 0)) != hipSuccess) return err;
        hipLaunchKernelGGL(mt_table_kernel, dim3((unsigned)(e1 - e0)), dim3(256), mt_table_lds(R, st.m), ax->s,
                           st.mtpar, st, R, e0);
        if ((err = hipGetLastError()) != hipSuccess) return err;
    }
    if ((err = hipEventRecord(ax->ev[K], ax->s)) != hipSuccess) return err;
    return hipStreamWaitEvent(s, ax->ev[K], 0);
}

hipError_t launch_step(const asg_batch_view &bv, const EnvState &st, int ts, int k, hipStream_t s, bool assign_ready) {
    if (st.mtpar) return launch_step_src(par_src(st), bv, st, ts, k, s, assign_ready);
    if (uses_table(st)) return launch_step_src(table_src(st), bv, st, ts, k, s, assign_ready);
    return launch_step_src(bump_src(st), bv, st, ts, k, s, assign_ready);
}

template <class Src>
static hipError_t launch_random_rollout_src(const Src &src, const asg_batch_view &bv, const EnvState &st, int ts,
                                            int k0, int steps, bool reset, hipStream_t s) {
    const size_t lds = sizeof(int) * (size_t)(2 * st.n + 2 * st.m + 2) + sizeof(double) * st.n + 16;
    // one wave per 64 work items of the row writer (VEC tasks each), at most 4 waves
    const int64_t items = (int64_t)st.n * ((st.m + 3) / 4);
    const int threads = items >= 256 ? 256 : (int)((items + 63) / 64 * 64);
    if (vec4_ok(bv, st.m))
        hipLaunchKernelGGL((random_rollout_kernel<4, Src>), dim3(st.E), dim3(threads), lds, s, src, bv, st, ts, k0, steps,
                           reset ? 1 : 0);
    else
        hipLaunchKernelGGL((random_rollout_kernel<1, Src>), dim3(st.E), dim3(threads), lds, s, src, bv, st, ts, k0, steps,
                           reset ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_random_rollout(const asg_batch_view &bv, const EnvState &st, int ts, int k0, int steps, bool reset,
                                 hipStream_t s) {
    if (st.mtpar) return launch_random_rollout_src(par_src(st), bv, st, ts, k0, steps, reset, s);
    if (uses_table(st)) return launch_random_rollout_src(table_src(st), bv, st, ts, k0, steps, reset, s);
    return launch_random_rollout_src(bump_src(st), bv, st, ts, k0, steps, reset, s);
}

hipError_t launch_random_actions(const asg_batch_view &bv, const EnvState &st, int ts, int k, hipStream_t s) {
    hipLaunchKernelGGL(random_actions_kernel, dim3(st.E), dim3(64), 0, s, bv, st, ts, k);
    return hipGetLastError();
}

hipError_t launch_export_bump_params(const EnvState &st, float *out, hipStream_t s) {
    hipLaunchKernelGGL(export_bump_params_kernel, dim3(st.E), dim3(256), sizeof(float) * st.m, s, bump_src(st), st,
                       out);
    return hipGetLastError();
}

hipError_t launch_export_table(const EnvState &st, double *out, hipStream_t s) {
    const size_t lds = sizeof(float) * st.m + 16;
    if (st.mtpar)
        hipLaunchKernelGGL((export_table_kernel<ParSrc>), dim3(st.E), dim3(256), lds, s, par_src(st), st, out);
    else if (uses_table(st))
        hipLaunchKernelGGL((export_table_kernel<TableSrc>), dim3(st.E), dim3(256), lds, s, table_src(st), st, out);
    else
        hipLaunchKernelGGL((export_table_kernel<BumpSrc>), dim3(st.E), dim3(256), lds, s, bump_src(st), st, out);
    return hipGetLastError();
}

hipError_t launch_import_table(const double *in, int64_t src_envs, const EnvState &st, hipStream_t s) {
    hipLaunchKernelGGL(import_table_kernel, dim3(st.E), dim3(256), 0, s, in, st, st.table, src_envs);
    return hipGetLastError();
}

hipError_t launch_export_prev(const EnvState &st, int64_t *out, hipStream_t s) {
    hipLaunchKernelGGL(export_prev_kernel, dim3(st.E), dim3(64), 0, s, st, out);
    return hipGetLastError();
}

hipError_t launch_mt_seed(const EnvState &st, hipStream_t s) {
    const int64_t blocks = (st.E + 63) / 64;
    hipLaunchKernelGGL(mt_seed_kernel, dim3(blocks), dim3(64), 0, s, st.mt, st.E, st.seed, st.env_base,
                       (st.quirks & ASG_QUIRK_REPLICATE_STREAM) != 0);
    return hipGetLastError();
}

hipError_t launch_mt_advance(const EnvState &st, int64_t words, hipStream_t s) {
    hipLaunchKernelGGL(mt_advance_kernel, dim3(st.E), dim3(64), sizeof(uint32_t) * 2 * kMtN, s, st.mt, words);
    return hipGetLastError();
}

}  // namespace asg
