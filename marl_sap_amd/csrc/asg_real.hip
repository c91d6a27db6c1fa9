// asg_real.hip -- batched RealConstellationEnv, constant-benefit
// path (injected sat_prox_mat, the only one that runs without the orbital simulator).
//
// Reference: src/envs/real_constellation_env.py.  Per env and step:
//   rewards   beta_hat[i, a_i, 0] / count(a_i) (or the full penalty), with
//             beta_hat[..., 0] = beta[..., 0] - lambda * T_trans[prev_i, j] * (sum_l beta > 1e-12)  (:135-158, :259-327)
//   beta      sat_prox_mat[:, :, k:k+L] * task_prios, zero past T                                       (:110, :164-168)
//   obs       per agent: its top-M tasks (L-deep benefits), the N agents competing hardest for them,
//             their benefits on those tasks and on their own top M/2 other tasks, and a
//             one-hot of its previous task among its top M                                             (:177-230)
// float64 arithmetic as numpy (the L-sum left to right), stored through float32 into
// the float16 / int16 scheme (real_constellation_env.py:80-97) like torch's casts.
// np.argsort's unspecified tie order is replaced by the stable order (lower index
// first), as in oracle/asg_real_oracle.c.
//
// Layout: the benefit table is stored time-major, table[e][k][i][j] (float64), so one
// step reads L contiguous [n][m] slices; env stride 0 = one table shared by all envs
// (the reference's constant-benefit mode).  Per step: a transition kernel (one workgroup
// per env: counts, rewards, returns), a strip kernel (one workgroup per S agents of an
// env: the pre-transition row, the L-summed totals kept in LDS and written task-major,
// each agent's ranked task lists), and an observation kernel (one wave per agent).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <algorithm>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../include/asg.h"
#include "asg_device.h"
#include "asg_internal.h"

#ifndef ASG_REAL_PROF_SKIP
#define ASG_REAL_PROF_SKIP 0  // profiling only: skip phases (wrong results)
#endif
namespace asg {

struct RealState {
    int64_t E;
    int n, m, T, L, N, M;
    double lambda_;
    const double *table;  // [E or 1][T][n][m]
    int64_t table_env_stride;
    const double *prios;    // [m]
    const double *T_trans;  // [m][m]
    int *prev;              // [E][n]
    double *returns;        // [E]
    float *totT;            // [E][m][n] L-summed totals of the current beta rounded to float32, task-major
    int *topA;              // [E][n][M]        each agent's top-M tasks, ties -> lower index
    int *topD;              // [E][n][M + M/2]  its top tasks, ties -> higher index
    int *err;
    int variant;            // asg_real_variant
    double *power;          // [E][n] power states (power / interference variants)
    const int *bands;       // [n] frequency band per satellite (interference)
    const double *nbr;      // [m][m] task neighbour matrix (interference)
    const int64_t *prev0;   // injected reset assignments [count][n] or nullptr (Philox)
    int64_t prev0_env_stride;
    uint64_t seed;
    int64_t env_base;
    uint32_t episode;
    int bids;                     // bids_as_actions: actions are float32 [n][m] bids
    const int64_t *assign;        // bids: LSA(bids row, maximize) assignments [E][n] of this step
    const int32_t *assign_status; // bids: their LSA status [E] (0, ASG_E_LSA_INVALID / _INFEASIBLE)
};

__device__ __forceinline__ void store_real(const asg_field &f, int64_t off, double v) {
    switch (f.dtype) {
        case ASG_F32: reinterpret_cast<float *>(f.ptr)[off] = (float)v; break;
        case ASG_F16: reinterpret_cast<__half *>(f.ptr)[off] = __float2half((float)v); break;
        case ASG_F64: reinterpret_cast<double *>(f.ptr)[off] = v; break;
        default: break;
    }
}
__device__ __forceinline__ void store_int(const asg_field &f, int64_t off, int64_t v) {
    switch (f.dtype) {
        case ASG_I64: reinterpret_cast<int64_t *>(f.ptr)[off] = v; break;
        case ASG_I32: reinterpret_cast<int32_t *>(f.ptr)[off] = (int32_t)v; break;
        case ASG_I16: reinterpret_cast<int16_t *>(f.ptr)[off] = (int16_t)v; break;
        case ASG_BOOL: reinterpret_cast<uint8_t *>(f.ptr)[off] = v != 0; break;
        default: break;
    }
}
__device__ __forceinline__ int64_t load_int(const asg_field &f, int64_t off) {
    switch (f.dtype) {
        case ASG_I64: return reinterpret_cast<const int64_t *>(f.ptr)[off];
        case ASG_I32: return reinterpret_cast<const int32_t *>(f.ptr)[off];
        case ASG_I16: return reinterpret_cast<const int16_t *>(f.ptr)[off];
        default: return 0;
    }
}
__device__ __forceinline__ int64_t foff(const asg_field &f, int64_t b, int64_t t, int64_t d2, int64_t d3) {
    return b * f.stride[0] + t * f.stride[1] + d2 * f.stride[2] + d3 * f.stride[3];
}

// beta value (i, j, l) at time k: table slice * task priority, zero past T
__device__ __forceinline__ double real_beta(const RealState &st, const double *tab, int k, int i, int j, int l) {
    const int kk = k + l;
    const double v = kk < st.T ? tab[((int64_t)kk * st.n + i) * st.m + j] : 0.0;
    return v * st.prios[j];
}

// wave-wide selection of the best remaining candidate: value order descending, ties to the
// lower index (HIGHER_TIES = false, np.argsort(-x) stable) or to the higher index
// (HIGHER_TIES = true: the tail of an ascending stable argsort)
template <bool HIGHER_TIES, class V = double>
__device__ __forceinline__ int wave_select(const V *vals, unsigned char *taken, int len) {
    const int lane = threadIdx.x & 63;
    V bv = -INFINITY;
    int bj = -1;
    for (int j = lane; j < len; j += 64) {
        if (taken[j]) continue;
        const V v = vals[j];
        const bool better = bj < 0 || v > bv || (v == bv && (HIGHER_TIES ? j > bj : j < bj));
        if (better) {
            bv = v;
            bj = j;
        }
    }
    const V vmax = wave_allreduce(bj >= 0 ? bv : (V)-INFINITY, [](V a, V b) { return a > b ? a : b; });
    int key;
    if (HIGHER_TIES) {
        key = wave_max_i32(bj >= 0 && bv == vmax ? bj : -1);
    } else {
        key = -wave_max_i32(bj >= 0 && bv == vmax ? -bj : -0x7fffffff);
    }
    return key;
}

// Top-K of vals[0..len) in the same order as K successive wave_select calls, for short
// lists (len <= 64 * CAP; vals in LDS): every lane sorts its own CAP candidates
// (j = lane + 64 c) once, then keeps only their indices.  Each pick reads the lanes' list
// heads back from LDS and reduces float32-rounded keys (one DPP-fused max): rounding is
// monotone, so a unique maximal key is the unique float64 maximum; equal keys take the
// exact path (float64 compare against the first candidate, then the index rule).  The
// winning lane shifts its index list -- no rescans.  (V = float: the keys are the values.)
// The picks go out 64 at a time, lane k holding pick k (one store instead of one per pick);
// the return value is lane k's pick k for k < min(K, 64) (-1 past K).  (Keeping float32
// values in registers beside the indices instead of re-reading them measured no faster.)
#ifndef ASG_TOPK_NET8
#define ASG_TOPK_NET8 1
#endif
template <int CAP, bool HIGHER_TIES, class V = double>
__device__ __forceinline__ int wave_topk_heads(const V *vals, int len, int K, int *out) {
    const int lane = threadIdx.x & 63;
    int id[CAP];
    {
        V v[CAP];
#pragma unroll
        for (int c = 0; c < CAP; ++c) {
            const int j = lane + 64 * c;
            v[c] = j < len ? vals[j] : -INFINITY;
            id[c] = j < len ? j : -1;  // -1: no candidate (sorts last, never wins)
        }
        auto before = [](V va, int ia, V vb, int ib) {
            if (ia < 0) return false;
            if (ib < 0) return true;
            return va > vb || (va == vb && (HIGHER_TIES ? ia > ib : ia < ib));
        };
        auto cswap = [&](int a, int b) {  // a < b: a gets the one that comes first
            if (before(v[b], id[b], v[a], id[a])) {
                const V tv = v[a];
                v[a] = v[b];
                v[b] = tv;
                const int ti = id[a];
                id[a] = id[b];
                id[b] = ti;
            }
        };
        if constexpr (CAP == 6 && ASG_TOPK_NET8) {  // the 12-comparator network for 6 inputs
            constexpr int kNet6[12][2] = {{0, 5}, {1, 3}, {2, 4}, {1, 2}, {3, 4}, {0, 3},
                                          {2, 5}, {0, 1}, {2, 3}, {4, 5}, {1, 2}, {3, 4}};
#pragma unroll
            for (int q = 0; q < 12; ++q) cswap(kNet6[q][0], kNet6[q][1]);
        } else if constexpr (CAP == 8 && ASG_TOPK_NET8) {
            // the 19-comparator sorting network for 8 inputs (depth 6) in place of the
            // 28-comparator odd-even transposition sort: same order (a total order on (value, index))
            constexpr int kNet[19][2] = {{0, 2}, {1, 3}, {4, 6}, {5, 7}, {0, 4}, {1, 5}, {2, 6}, {3, 7}, {0, 1}, {2, 3},
                                         {4, 5}, {6, 7}, {2, 4}, {3, 5}, {1, 4}, {3, 6}, {1, 2}, {3, 4}, {5, 6}};
#pragma unroll
            for (int q = 0; q < 19; ++q) cswap(kNet[q][0], kNet[q][1]);
        } else {
#pragma unroll
            for (int pass = 0; pass < CAP; ++pass)  // odd-even transposition sort, fully unrolled
#pragma unroll
                for (int c = pass & 1; c + 1 < CAP; c += 2) cswap(c, c + 1);
        }
    }
    int mine = -1, first = -1;
    for (int k = 0; k < K; ++k) {
        const bool has = id[0] >= 0;
        const V x = has ? vals[id[0]] : (V)-INFINITY;
        const float key = has ? (float)x : -INFINITY;
        const float kmax = wave_max_f32_nonan(key);
        uint64_t cm = __ballot(has && key == kmax);
        // NaN totals (an injected NaN benefit) match no key: rank them last, by index, so
        // every pick stays a valid task index
        if (cm == 0) cm = __ballot(has);
        int wl = (int)__builtin_ctzll(cm);  // winning lane
        if (__popcll(cm) != 1) {
            // equal keys: exact float64 maximum among them, then the index rule
            V vmax;
            if constexpr (sizeof(V) == 8) {
                const uint64_t xb = __builtin_bit_cast(uint64_t, x);
                const uint32_t lo0 = __builtin_amdgcn_readlane((int)(uint32_t)xb, wl);
                const uint32_t hi0 = __builtin_amdgcn_readlane((int)(uint32_t)(xb >> 32), wl);
                vmax = __builtin_bit_cast(V, (uint64_t)lo0 | ((uint64_t)hi0 << 32));
            } else {
                vmax = __builtin_bit_cast(V, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), wl));
            }
            uint64_t cand = cm;
            if ((__ballot(x != vmax) & cm) != 0) {
                const bool in = __builtin_amdgcn_inverse_ballot_w64(cm);
                vmax = wave_allreduce(in ? x : (V)-INFINITY, [](V a, V b) { return a > b ? a : b; });
                cand = __ballot(x == vmax) & cm;
            }
            if (cand == 0) cand = cm;  // NaN maximum: the index rule over all candidates
            const bool cb = __builtin_amdgcn_inverse_ballot_w64(cand);
            const int win = HIGHER_TIES ? wave_max_i32(cb ? id[0] : -1) : -wave_max_i32(cb ? -id[0] : -0x7fffffff);
            wl = (int)__builtin_ctzll(__ballot(has && id[0] == win));
        }
        const int win = __builtin_amdgcn_readlane(id[0], wl);
        if (lane == (k & 63)) mine = win;
        if ((k & 63) == 63 || k == K - 1) {
            if (lane <= (k & 63)) out[(k & ~63) + lane] = mine;
            if (k < 64) first = mine;
        }
        if (lane == wl) {
#pragma unroll
            for (int c = 0; c + 1 < CAP; ++c) id[c] = id[c + 1];
            id[CAP - 1] = -1;
        }
    }
    return K > 0 ? first : -1;
}

// top-K: register heads when len <= 64 * CAP (CAP > 0, chosen per kernel instance so each
// gets its own register budget), else K rescans (CAP = 0; taken: [len] scratch)
template <int CAP, bool HIGHER_TIES, class V = double>
__device__ __forceinline__ void wave_topk(const V *vals, int len, int K, int *out, unsigned char *taken) {
    if constexpr (CAP > 0) {
        (void)wave_topk_heads<CAP, HIGHER_TIES, V>(vals, len, K, out);
    } else {
        const int lane = threadIdx.x & 63;
        for (int j = lane; j < len; j += 64) taken[j] = 0;
        wave_sync();
        for (int c = 0; c < K; ++c) {
            const int j = wave_select<HIGHER_TIES, V>(vals, taken, len);
            if (lane == 0) {
                out[c] = j;
                taken[j] = 1;
            }
            wave_sync();
        }
    }
    wave_sync();
}

// ---- one step's rewards and power update of one env (block-wide; every thread calls) -----
// The variants' reward rules, shared by the transition kernel and HAAL's sequence values:
//   plain / power  beta_hat[i, a_i, 0] / count(a_i), or the full penalty when beta_hat <= 0
//                  (real_constellation_env.py:145-160); power: 0 for a dead satellite, beta_hat
//                  zeroed below 1e-12 power (real_power_constellation_env.py:150-165, :343-347)
//   interference   beta[i, a_i, 0] * 0.5 ** conflicts / count over applicable agents, minus
//                  lambda on a handover (interference_constellation_env.py:309-353)
// sa [n] this step's tasks, prevp(i) the previous task of agent i, pw [n] power (power
// variants), LDS scnt [m], sapp [n]; rewards into srew [n].
template <class PrevF>
__device__ __forceinline__ void real_step_rewards(const RealState &st, const double *tab, int k, const int *sa,
                                                  PrevF prevp, const double *pw, int *scnt, int *sapp,
                                                  double *srew) {
    const int n = st.n, m = st.m, L = st.L;
    for (int j = threadIdx.x; j < m; j += blockDim.x) scnt[j] = 0;
    __syncthreads();
    if (st.variant == ASG_REAL_INTERFERENCE) {
        // applicable = alive and on a meaningful task; counts over applicable agents only
        for (int i = threadIdx.x; i < n; i += blockDim.x)
            sapp[i] = (pw[i] <= 0 ? 0 : 1) * (real_beta(st, tab, k, i, sa[i], 0) < 1e-12 ? 0 : 1);
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += blockDim.x)
            if (sapp[i]) atomicAdd(&scnt[sa[i]], 1);
    } else {
        for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&scnt[sa[i]], 1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int c = sa[i];
        const int pv = prevp(i);
        double r;
        if (st.variant == ASG_REAL_INTERFERENCE) {
            // conflicts = sum over the agents of i's band of nbr[a_i, a_j] * applicable_j - 1
            // (interference_constellation_env.py:327-331), then 0.5 ** conflicts
            double conf = 0.0;
            const int band = st.bands[i];
            for (int a = 0; a < n; ++a)
                if (st.bands[a] == band) conf = conf + st.nbr[(int64_t)c * m + sa[a]] * (double)sapp[a];
            conf = conf - 1.0;
            r = real_beta(st, tab, k, i, c, 0) * pow(0.5, conf);
            if (scnt[c] > 0) r = r / (double)scnt[c];
            if (sapp[i] && pv != c) r = r - st.lambda_;
        } else if (st.variant == ASG_REAL_POWER && !(pw[i] > 0)) {
            r = 0.0;  // dead satellite (real_power_constellation_env.py:161-162)
        } else {
            double bh;
            if (st.variant == ASG_REAL_POWER && pw[i] < 1e-12) {
                bh = 0.0;  // beta_hat zeroed below 1e-12 power (:343-347)
            } else {
                double s = real_beta(st, tab, k, i, c, 0);
                const double b0 = s;
                for (int l = 1; l < L; ++l) s = s + real_beta(st, tab, k, i, c, l);
                const double cond = s > 1e-12 ? 1.0 : 0.0;
                const double pen = st.T_trans[(int64_t)pv * m + c] * cond;
                bh = b0 - st.lambda_ * pen;
            }
            r = bh > 0 ? bh / (double)scnt[c] : bh;
        }
        srew[i] = r;
    }
}

// power update on the pre-step beta (real_power_constellation_env.py:170-178); the caller
// syncs before (every reader of the old power is done)
__device__ __forceinline__ void real_power_update(const RealState &st, const double *tab, int k, const int *sa,
                                                  double *pw) {
    for (int i = threadIdx.x; i < st.n; i += blockDim.x)
        if (pw[i] > 0) {
            if (real_beta(st, tab, k, i, sa[i], 0) > 1e-12) {
                pw[i] -= 0.2;
            } else {
                const double p = pw[i] + 0.1;
                pw[i] = p < 1.0 ? p : 1.0;
            }
        }
}

// ---- kernel 1: the transition of each env (step only), one workgroup per env ---------------
// LDS: actions [n] int, counts [m] int, rewards [n] f64, applicable [n] int
__host__ __device__ __forceinline__ size_t transition_lds(int n, int m) {
    return (size_t)4 * (n + m + 1) + 8 * (size_t)n + 8 + 4 * (size_t)n;  // + applicable [n]
}

__global__ void __launch_bounds__(256) real_transition_kernel(asg_batch_view bv, RealState st, int ts, int k) {
    extern __shared__ unsigned char s_raw[];
    const int64_t e = blockIdx.x;
    const int n = st.n, m = st.m;
    int *sa = reinterpret_cast<int *>(s_raw);                                        // [n]
    int *scnt = sa + n;                                                              // [m]
    double *srew = reinterpret_cast<double *>(scnt + m + (((n + m) & 1) ? 1 : 0));  // [n], 8-B aligned
    const double *tab = st.table + e * st.table_env_stride;
    int *prev = st.prev + e * n;
    const int lsa_st = st.assign ? st.assign_status[e] : 0;
    if (lsa_st != 0 && threadIdx.x == 0) atomicCAS(st.err, 0, lsa_st);  // scipy's ValueError
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        // bids_as_actions: the assignments of LSA(bids, maximize) (real_constellation_env.py:
        // 140-142, real_power_constellation_env.py:142, interference_constellation_env.py:159)
        int64_t a = st.assign ? (lsa_st != 0 ? 0 : st.assign[e * n + i]) : load_int(bv.actions, foff(bv.actions, e, ts, i, 0));
        if (a < 0 || a >= m) {
            atomicCAS(st.err, 0, ASG_E_ACTION_RANGE);
            a = a < 0 ? 0 : m - 1;
        }
        sa[i] = (int)a;
    }
    double *pw = st.power + e * n;
    int *sapp = reinterpret_cast<int *>(srew + n);  // [n] applicable (interference)
    real_step_rewards(st, tab, k, sa, [&](int i) { return prev[i]; }, pw, scnt, sapp, srew);
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        if (bv.rewards.ptr) store_real(bv.rewards, foff(bv.rewards, e, ts, i, 0), srew[i]);
    if (st.variant != ASG_REAL_PLAIN) {
        __syncthreads();  // every reader of the old power is done
        real_power_update(st, tab, k, sa, pw);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double tot = 0.0;
        for (int i = 0; i < n; ++i) tot += srew[i];  // Python sum(rewards), left to right
        st.returns[e] += tot;
        if (bv.terminated.ptr) store_int(bv.terminated, foff(bv.terminated, e, ts, 0, 0), k + 1 >= st.T);
    }
    for (int i = threadIdx.x; i < n; i += blockDim.x) prev[i] = sa[i];
}

// ---- reset: assignments, power, returns (one workgroup per env) -------------------------
//   plain:          prev_assigns = arange(n)                              (:111)
//   power variants: np.random.choice(m, n, replace=False) -- the injected assignments, or a
//                   Philox Fisher-Yates keyed (seed, global env, episode) -- and full power
__global__ void __launch_bounds__(256) real_reset_kernel(RealState st) {
    extern __shared__ int s_perm[];
    const int64_t e = blockIdx.x;
    const int n = st.n, m = st.m;
    int *prev = st.prev + e * n;
    if (st.variant == ASG_REAL_PLAIN) {
        for (int i = threadIdx.x; i < n; i += blockDim.x) prev[i] = i;
    } else if (st.prev0) {
        const int64_t *p0 = st.prev0 + e * st.prev0_env_stride;
        for (int i = threadIdx.x; i < n; i += blockDim.x) prev[i] = (int)p0[i];
    } else {
        for (int j = threadIdx.x; j < m; j += blockDim.x) s_perm[j] = j;
        __syncthreads();
        if (threadIdx.x == 0) {
            const EnvKey key = env_key(st.seed, st.env_base + e);
            for (int i = m - 1; i >= 1; --i) {
                const u32x4 r = philox4x32_10(u32x4{(uint32_t)i, 0u, kCtrPerm, st.episode}, key.k0, key.k1);
                const int jj = (int)(((uint64_t)r.x * (uint64_t)(i + 1)) >> 32);
                const int t = s_perm[i];
                s_perm[i] = s_perm[jj];
                s_perm[jj] = t;
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += blockDim.x) prev[i] = s_perm[i];
    }
    for (int i = threadIdx.x; i < n; i += blockDim.x) st.power[e * n + i] = 1.0;
    if (threadIdx.x == 0) st.returns[e] = 0.0;
}

// ---- kernel 2: the pre-transition row and each agent's task ranking, one workgroup per
// strip of S agents of one env --------------------------------------------------------
// Writes beta (float16 [n][m][L]), avail, prev_assigns, filled (and, after a step, the
// one-hot of the actions at row ts); keeps the strip's L-summed totals in LDS, writes
// them task-major rounded to float32 (totT, coalesced per task across the strip; the
// observation pass's competitor prefilter) and ranks each agent's row:
//   topA[a] = the M best tasks, ties to the lower index      (np.argsort(-total)[:M], :192)
//   topD[a] = the M + M/2 best tasks, ties to the higher index (the order of the tail of
//             np.argsort(row)[:, -M//2:], :212-214); an agent's M/2 best tasks outside
//             any M-task set are always among them (m >= M + M/2 is required)
// LDS: totals [S][m] f64, then one `taken` byte row per wave (64 * S threads = S waves)
__host__ __device__ __forceinline__ size_t strip_lds(int S, int m) {
    return (size_t)S * m * 8 + (size_t)S * ((m + 3) & ~3);
}

// the strip's grouped-load path: kStripJG task iterations (of 64) per load group, L <= kStripLM
#ifndef ASG_STRIP_JG
#define ASG_STRIP_JG 1
#endif
#ifndef ASG_STRIP_GROUPED
#define ASG_STRIP_GROUPED 1
#endif
#ifndef ASG_OBS_TWOPHASE
#define ASG_OBS_TWOPHASE 1
#endif
constexpr int kStripJG = ASG_STRIP_JG, kStripLM = 3;
// the deferred-store path (m <= 64 kStripIt, L <= kStripLM): the whole row is loaded (two task
// iterations in flight) and reduced into registers -- float16 beta packed, the totals in LDS --
// before any of its global stores, so no load waits behind a store's acknowledgement
#ifndef ASG_STRIP_DEFER
#define ASG_STRIP_DEFER 1
#endif
constexpr int kStripIt = 8;
// ASG_STRIP_WAVES: waves per SIMD the strip kernel is compiled for (0: the allocator's choice).
// 8 (64 VGPRs, a few spills outside the row loop) measured 1.69 ms per real step at E = 512 against
// 1.83 at 7 waves and 1.90 at the allocator's 80 VGPRs (profiles/r6_real_ab_s8.txt)
#ifndef ASG_STRIP_WAVES
#define ASG_STRIP_WAVES 8
#endif
// a buffer descriptor the compiler can prove wave-uniform (base and size through readfirstlane)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void *p, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>((uint64_t)lo | ((uint64_t)hi << 32)), 0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
template <int CAP>
__global__ void __launch_bounds__(1024)
#if ASG_STRIP_WAVES
__attribute__((amdgpu_waves_per_eu(CAP >= 16 ? 4 : ASG_STRIP_WAVES)))  // (CAP 16: m > 512, registers first)
#endif
real_strip_kernel(asg_batch_view bv, asg_field pfield, RealState st, int ts,
                                                          int knew, int step, int S) {
    extern __shared__ unsigned char s_raw[];
    const int n = st.n, m = st.m, L = st.L, M = st.M, MD = st.M + st.M / 2;
    const int64_t e = blockIdx.y;
    const int i0 = blockIdx.x * S;
    const int rows = n - i0 < S ? n - i0 : S;
    double *tl = reinterpret_cast<double *>(s_raw);                        // [S][m] totals
    unsigned char *taken_all = s_raw + (size_t)S * m * 8;                   // [S waves][m]
    const double *tab = st.table + e * st.table_env_stride;
    int *prev = st.prev + e * n;
    const int row = step ? ts + 1 : ts;
    // one wave per agent row of the strip, lanes along the tasks: per row the field bases
    // are computed once; the scheme's own dtypes (f16 beta, bool avail, i16 one-hot) take
    // typed stores, anything else the generic ones
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, waves = blockDim.x >> 6;
    // (bids_as_actions: no actions_onehot field -- the scheme has no preprocess, :110-112)
    const bool fast = bv.beta.dtype == ASG_F16 && bv.avail_actions.dtype == ASG_BOOL &&
                      (!step || !bv.actions_onehot.ptr || bv.actions_onehot.dtype == ASG_I16) && bv.beta.ptr &&
                      bv.avail_actions.ptr;
    for (int r = wave; r < rows; r += waves) {
        const int i = i0 + r;
        const double *t0 = tab + ((int64_t)knew * n + i) * m;  // slice knew, row i
        const int64_t slice = (int64_t)n * m;
        int eff = st.T - knew < L ? st.T - knew : L;
        eff = eff < 0 ? 0 : eff;
        const int pa = prev[i];
        double *trow = tl + (int64_t)r * m;
        if (ASG_STRIP_DEFER && fast && L == 3 && m <= 64 * kStripIt && bv.beta.stride[3] == 3 &&
            bv.avail_actions.stride[3] == 1 && (!step || !bv.actions_onehot.ptr || bv.actions_onehot.stride[3] == 1)) {
            // buffer descriptors over the row's slices and fields: 32-bit lane offsets, and the
            // range check zeroes the loads (and drops the stores) of tasks past m and of slices
            // past the episode end -- every memory instruction below is unconditional
            const bool oh = step && bv.actions_onehot.ptr;
            __amdgpu_buffer_rsrc_t rs[kStripLM];
#pragma unroll
            for (int l = 0; l < kStripLM; ++l) rs[l] = uniform_rsrc(t0 + l * slice, l < eff ? (uint32_t)m * 8u : 0u);
            const __amdgpu_buffer_rsrc_t rp = uniform_rsrc(st.prios, (uint32_t)m * 8u);
            double va[kStripLM], vb[kStripLM], pra, prb;
            const uint32_t off = 8u * (uint32_t)lane;
            auto issue = [&](double (&v)[kStripLM], double &pr, int it) {  // iteration it: + 512 it bytes
                pr = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rp, off, 512 * it, 0));
#pragma unroll
                for (int l = 0; l < kStripLM; ++l)
                    v[l] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs[l], off, 512 * it, 0));
            };
            uint32_t pk0[kStripIt], pk1[kStripIt];  // float16 beta: l0 | l1 << 16, l2
            auto reduce = [&](const double (&v)[kStripLM], double pr, int it) {
                const int j = 64 * it + lane;
                double sum = 0.0;
                uint32_t h[kStripLM];
#pragma unroll
                for (int l = 0; l < kStripLM; ++l) {
                    const double b = v[l] * pr;  // (a zeroed slice: 0 * pr, as l >= eff reads 0)
                    if (l < L) sum = l == 0 ? b : sum + b;
                    h[l] = __half_as_ushort(__float2half((float)b));
                }
                if (j < m) trow[j] = sum;
                pk0[it] = h[0] | (h[1] << 16);
                pk1[it] = h[2];
                // materialise the packed halves here: otherwise the conversions sink to the stores
                // and the three float64 products of every iteration stay live until then
                asm volatile("" : "+v"(pk0[it]), "+v"(pk1[it]));
            };
            issue(va, pra, 0);
#pragma unroll
            for (int it = 0; it < kStripIt; it += 2) {
                issue(vb, prb, it + 1);
                reduce(va, pra, it);
                if (it + 2 < kStripIt) issue(va, pra, it + 2);
                reduce(vb, prb, it + 1);
            }
            if (!(ASG_REAL_PROF_SKIP & 2)) {
                const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(
                    reinterpret_cast<__half *>(bv.beta.ptr) + foff(bv.beta, e, row, i, 0), 6u * (uint32_t)m);
                const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(
                    reinterpret_cast<uint8_t *>(bv.avail_actions.ptr) + foff(bv.avail_actions, e, row, i, 0), (uint32_t)m);
                const __amdgpu_buffer_rsrc_t ro = uniform_rsrc(
                    oh ? reinterpret_cast<int16_t *>(bv.actions_onehot.ptr) + foff(bv.actions_onehot, e, ts, i, 0)
                       : nullptr,
                    oh ? 2u * (uint32_t)m : 0u);
                // beta: 6 bytes per task at 2-byte alignment -> one dword + one short; task j = 64 it
                // + lane starts at byte 384 it + 6 lane, so the alignment is the lane's for every
                // iteration and the iteration is an immediate offset
                const uint32_t base_odd = (uint32_t)(reinterpret_cast<uintptr_t>(bv.beta.ptr) +
                                                     2 * foff(bv.beta, e, row, i, 0)) & 2u;
                const bool al = ((6u * (uint32_t)lane + base_odd) & 3u) == 0u;
                const uint32_t odw = 6u * (uint32_t)lane + (al ? 0u : 2u), osh = 6u * (uint32_t)lane + (al ? 4u : 0u);
#pragma unroll
                for (int it = 0; it < kStripIt; ++it) {
                    const uint32_t h0 = pk0[it] & 0xffffu, h1 = pk0[it] >> 16, h2 = pk1[it];
                    __builtin_amdgcn_raw_buffer_store_b32(al ? pk0[it] : (h1 | (h2 << 16)), rb, odw, 384 * it, 0);
                    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(al ? h2 : h0), rb, osh, 384 * it, 0);
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)1, ra, (uint32_t)lane, 64 * it, 0);
                    if (oh)
                        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(pa == 64 * it + lane), ro, 2u * (uint32_t)lane,
                                                              128 * it, 0);
                }
            }
        } else if (ASG_STRIP_GROUPED && fast && L <= kStripLM) {
            // the row's table values in groups of kStripJG task iterations: every load of a group
            // (the L slices and the priorities) is issued before the group's stores -- gfx9 retires
            // loads and stores in order, so a load issued behind a store waits for its acknowledgement
            __half *bb = reinterpret_cast<__half *>(bv.beta.ptr) + foff(bv.beta, e, row, i, 0);
            uint8_t *ab = reinterpret_cast<uint8_t *>(bv.avail_actions.ptr) + foff(bv.avail_actions, e, row, i, 0);
            int16_t *ob = step && bv.actions_onehot.ptr
                              ? reinterpret_cast<int16_t *>(bv.actions_onehot.ptr) + foff(bv.actions_onehot, e, ts, i, 0)
                              : nullptr;
            const int64_t bs3 = bv.beta.stride[3], as3 = bv.avail_actions.stride[3];
            const int64_t os3 = ob ? bv.actions_onehot.stride[3] : 0;
            for (int jb = 0; jb < m; jb += 64 * kStripJG) {
                double v[kStripJG][kStripLM], pr[kStripJG];
#pragma unroll
                for (int g = 0; g < kStripJG; ++g) {
                    const int j = jb + 64 * g + lane;
                    pr[g] = j < m ? st.prios[j] : 0.0;
#pragma unroll
                    for (int l = 0; l < kStripLM; ++l) v[g][l] = (j < m && l < eff) ? t0[l * slice + j] : 0.0;
                }
#pragma unroll
                for (int g = 0; g < kStripJG; ++g) {
                    const int j = jb + 64 * g + lane;
                    if (j >= m) continue;
                    double sum = 0.0;
#pragma unroll
                    for (int l = 0; l < kStripLM; ++l) {
                        if (l >= L) break;
                        const double b = v[g][l] * pr[g];
                        sum = l == 0 ? b : sum + b;
                        if (!(ASG_REAL_PROF_SKIP & 2)) bb[j * bs3 + l] = __float2half((float)b);
                    }
                    trow[j] = sum;
                    if (!(ASG_REAL_PROF_SKIP & 2)) {
                        ab[j * as3] = 1;
                        if (ob) ob[j * os3] = (int16_t)(pa == j);
                    }
                }
            }
        } else if (fast) {
            __half *bb = reinterpret_cast<__half *>(bv.beta.ptr) + foff(bv.beta, e, row, i, 0);
            uint8_t *ab = reinterpret_cast<uint8_t *>(bv.avail_actions.ptr) + foff(bv.avail_actions, e, row, i, 0);
            int16_t *ob = step && bv.actions_onehot.ptr
                              ? reinterpret_cast<int16_t *>(bv.actions_onehot.ptr) + foff(bv.actions_onehot, e, ts, i, 0)
                              : nullptr;
            const int64_t bs3 = bv.beta.stride[3], as3 = bv.avail_actions.stride[3];
            const int64_t os3 = ob ? bv.actions_onehot.stride[3] : 0;
            for (int j = lane; j < m; j += 64) {
                const double pr = st.prios[j];
                double sum = 0.0;
                for (int l = 0; l < L; ++l) {
                    const double b = (l < eff ? t0[l * slice + j] : 0.0) * pr;
                    sum = l == 0 ? b : sum + b;
                    if (!(ASG_REAL_PROF_SKIP & 2)) bb[j * bs3 + l] = __float2half((float)b);
                }
                trow[j] = sum;
                if (!(ASG_REAL_PROF_SKIP & 2)) {
                    ab[j * as3] = 1;
                    if (ob) ob[j * os3] = (int16_t)(pa == j);
                }
            }
        } else {
            for (int j = lane; j < m; j += 64) {
                double sum = 0.0;
                for (int l = 0; l < L; ++l) {
                    const double b = real_beta(st, tab, knew, i, j, l);
                    sum = l == 0 ? b : sum + b;
                    if (bv.beta.ptr) store_real(bv.beta, foff(bv.beta, e, row, i, j) + l, b);
                }
                trow[j] = sum;
                if (bv.avail_actions.ptr) store_int(bv.avail_actions, foff(bv.avail_actions, e, row, i, j), 1);
                if (step && bv.actions_onehot.ptr)
                    store_int(bv.actions_onehot, foff(bv.actions_onehot, e, ts, i, j), pa == j);
            }
        }
    }
    if (bv.prev_assigns.ptr)
        for (int r = threadIdx.x; r < rows; r += blockDim.x)
            store_int(bv.prev_assigns, foff(bv.prev_assigns, e, row, i0 + r, 0), prev[i0 + r]);
    if (pfield.ptr && st.variant != ASG_REAL_PLAIN)
        for (int r = threadIdx.x; r < rows; r += blockDim.x)
            store_real(pfield, foff(pfield, e, row, i0 + r, 0), st.power[e * n + i0 + r]);
    if (blockIdx.x == 0 && threadIdx.x == 0 && bv.filled.ptr) store_int(bv.filled, foff(bv.filled, e, row, 0, 0), 1);
    __syncthreads();
    if (knew >= st.T) return;  // done: no observation pass follows
    float *totT = st.totT + e * (int64_t)n * m;
    for (int64_t p = threadIdx.x; p < (int64_t)rows * m; p += blockDim.x) {
        const int j = (int)(p / rows), r = (int)(p - (int64_t)j * rows);
        totT[(int64_t)j * n + i0 + r] = (float)tl[(int64_t)r * m + j];
    }
    // rank each agent row of the strip, one wave per row
    unsigned char *taken = taken_all + (size_t)wave * ((m + 3) & ~3);
    for (int r = wave; r < rows; r += waves) {
        const double *vals = tl + (int64_t)r * m;
        const int a = i0 + r;
        if (ASG_REAL_PROF_SKIP & 1) {  // profiling: valid placeholder lists (tasks 0..)
            for (int c = lane; c < MD; c += 64) {
                if (c < M) st.topA[(e * n + a) * (int64_t)M + c] = c;
                st.topD[(e * n + a) * (int64_t)MD + c] = c;
            }
            continue;
        }
        int *outA = st.topA + (e * n + a) * (int64_t)M, *outD = st.topD + (e * n + a) * (int64_t)MD;
        if constexpr (CAP > 0) {
            // topD first; when its first M + 1 totals are strictly decreasing (no tie can reorder
            // or swap the M best: every other task is <= the (M+1)-th), topA is its first M
            if (MD <= 64) {
                const int d = wave_topk_heads<CAP, true>(vals, m, MD, outD);
                const double v = lane <= M && d >= 0 ? vals[d] : 0.0;
                const double vn = __shfl_down(v, 1);
                if (__ballot(lane < M && !(v > vn)) == 0) {
                    if (lane < M) outA[lane] = d;
                } else {
                    (void)wave_topk_heads<CAP, false>(vals, m, M, outA);
                }
                wave_sync();
                continue;
            }
        }
        wave_topk<CAP, false>(vals, m, M, outA, taken);
        wave_topk<CAP, true>(vals, m, MD, outD, taken);
    }
}

// ---- kernel 3: observation rows, one wave per agent ---------------------------------------
// per-wave LDS of the observation pass: best[n] f64, best32[n] f32, taken[n], top[max(M, 10)]
// (padded with top[0]), topn[N], oth[N][M/2], tmask[ceil(m / 32)] (agent i's top-M tasks as a bit
// set), slot[M + N M + N M/2] (the (agent, task) of each L-run of the row's benefit entries; in
// best32's place once the ranking is done, when it fits there -- at 324 x 450 that keeps a
// 4-wave workgroup under 20 KB, 8 per CU)
__host__ __device__ __forceinline__ size_t real_obs_lds_per_wave(int n, int m, int N, int M) {
    const int Mp = M > 10 ? M : 10;
    const int nsl = M + N * M + N * (M / 2);
    return ((size_t)n * 13 + 3 + 4 * (size_t)(Mp + N + N * (M / 2) + (m + 31) / 32 + (nsl > n ? nsl : 0)) + 15) &
           ~(size_t)15;
}

// Observation pass, one wave per (env, agent i): competitors from the task-major totals,
// their "other" tasks from topD, then the row (real_constellation_env.py:186-219).
// XCD-aware grid: workgroups are dealt round-robin over the 8 XCDs (block b runs on XCD
// b % 8), so block b serves env 8 * ((b / 8) / G) + b % 8: all G workgroups of an env
// land on one XCD and its [m][n] totals are fetched into one L2, not eight.
constexpr int kObsG = 16;  // observation entries per lane of the two-phase copy (obs_size <= 1024)
constexpr int kObsMD = 24; // topD list entries per competitor loaded at once (M + M/2 <= 24)
constexpr int kObsMB = 10; // top tasks per agent held in registers by the competitor scan (M <= 10)
#ifndef ASG_OBS_PIPE
#define ASG_OBS_PIPE 1
#endif
template <int CAP>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CAP >= 16 ? 4 : 8)))
real_obs_kernel(asg_batch_view bv, RealState st, int row, int knew, int G) {
    extern __shared__ unsigned char s_raw[];
    const int n = st.n, m = st.m, L = st.L, N = st.N, M = st.M, M2 = st.M / 2, MD = st.M + st.M / 2;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, waves = blockDim.x >> 6;
    const int64_t k = blockIdx.x / 8;
    const int64_t e = (int64_t)(blockIdx.x % 8) + 8 * (k / G);
    const int i = (int)(k % G) * waves + wave;
    if (e >= st.E || i >= n) return;
    const int osz = M * L + N * M * L + ((N * M) / 2) * L + M + (st.variant != ASG_REAL_PLAIN ? N + 1 : 0);
    if (knew >= st.T) {  // done: zero observations (:221-224)
        for (int p = lane; p < osz; p += 64) store_real(bv.obs, foff(bv.obs, e, row, i, 0) + p, 0.0);
        return;
    }
    const size_t per_wave = real_obs_lds_per_wave(n, m, N, M);
    unsigned char *base = s_raw + per_wave * wave;
    double *best = reinterpret_cast<double *>(base);                // [n]
    float *best32 = reinterpret_cast<float *>(base + 8 * (size_t)n);  // [n]
    unsigned char *taken = base + 12 * (size_t)n;                   // [n]
    int *top = reinterpret_cast<int *>(taken + ((n + 3) & ~3));  // [M]
    int *topn = top + (M > kObsMB ? M : kObsMB);                 // [N]
    int *oth = topn + N;                                         // [N][M2], ascending
    uint32_t *tmask = reinterpret_cast<uint32_t *>(oth + N * M2);  // [ceil(m / 32)]
    uint32_t *slot = M + N * M + N * M2 <= n ? reinterpret_cast<uint32_t *>(best32)  // [M + N M + N M2]
                                             : tmask + (m + 31) / 32;
    const int *myA = st.topA + (e * n + i) * (int64_t)M;
    const int pi = st.prev[e * n + i];  // (issued with the first load, used by the row's one-hot)
    for (int c = lane; c < M || c < kObsMB; c += 64) top[c] = myA[c < M ? c : 0];
    wave_sync();
    // (b) each agent's best total over agent i's top-M tasks, agent i excluded (:196-198), from
    //     the float32-rounded totals: rounding is monotone, so f32(x) < f32(y) implies x < y
    const float *totT = st.totT + e * (int64_t)n * m;
    const int Mb = (ASG_REAL_PROF_SKIP & 4) ? 1 : M;
    bool nan_seen = false;
    int a_done = 0;
    if (ASG_OBS_PIPE && Mb <= kObsMB) {
        // the rows of agent i's top tasks as wave-uniform (scalar) bases, lanes along the agents,
        // two 64-agent groups in flight: group t + 1's loads are issued before group t is reduced
        const float *rowp[kObsMB];
#pragma unroll
        for (int c = 0; c < kObsMB; ++c)
            rowp[c] = totT + (int64_t)__builtin_amdgcn_readfirstlane(top[c]) * n;  // (c >= M: the padding)
        // (every load unconditional -- rows past M repeat row top[0], groups past the last repeat
        // it -- so each reduce waits on a fixed count of the loads in flight)
        const int groups = (n + 63) >> 6;
        float va[kObsMB], vb[kObsMB];
        auto issue = [&](float (&v)[kObsMB], int g) {
            const int a = min(lane + 64 * min(g, groups - 1), n - 1);
#pragma unroll
            for (int c = 0; c < kObsMB; ++c) v[c] = rowp[c][a];
        };
        auto reduce = [&](const float (&v)[kObsMB], int g) {
            const int a = lane + 64 * g;
            float b = v[0];
            bool bad = b != b;
#pragma unroll
            for (int c = 1; c < kObsMB; ++c) {
                const bool on = c < Mb;
                bad |= on && v[c] != v[c];
                b = on && v[c] > b ? v[c] : b;
            }
            if (g < groups && a < n) {
                nan_seen |= bad;
                best32[a] = a == i ? -INFINITY : b;
                taken[a] = 0;
            }
        };
        issue(va, 0);
        for (int g = 0; g < groups; g += 2) {
            issue(vb, g + 1);
            reduce(va, g);
            issue(va, g + 2);
            reduce(vb, g + 1);
        }
        a_done = n;
    }
    for (int a = a_done + lane; a < n; a += 64) {
        float b = totT[(int64_t)top[0] * n + a];
        nan_seen |= b != b;
        for (int c = 1; c < Mb; ++c) {
            const float v = totT[(int64_t)top[c] * n + a];
            nan_seen |= v != v;
            b = v > b ? v : b;
        }
        best32[a] = a == i ? -INFINITY : b;
        taken[a] = 0;
    }
    wave_sync();
    const double *tab = st.table + e * st.table_env_stride;
    // (c) the N strongest competitors (np.argsort(-best)[:N]): ranked by the float32 keys; the
    //     float64 order is the same unless keys tie (among the N picks, or with the N-th) or are
    //     NaN -- then the exact float64 best of every agent whose key reaches the N-th pick's
    //     (any agent outside that set has N keys strictly above it) is recomputed from the table
    //     the way the strip summed it, the others are -inf, and the float64 ranking decides
    if (!(ASG_REAL_PROF_SKIP & 8)) {
        const bool anynan = __ballot(nan_seen) != 0;
        bool exact = anynan;
        float tau = -INFINITY;
        if (!exact) {
            wave_topk<CAP, false, float>(best32, n, N, topn, taken);
            tau = best32[topn[N - 1]];
            int ties = 0;
            for (int a = lane; a < n; a += 64) ties += best32[a] == tau;
            for (int q = lane; q + 1 < N; q += 64) ties += 2 * (best32[topn[q]] == best32[topn[q + 1]]);
            exact = wave_allreduce(ties, [](int x, int y) { return x + y; }) > 1;
        }
        if (exact) {
            auto total = [&](int a, int j) {  // the strip's L-sum of beta[a, j, :]
                double sum = 0.0;
                for (int l = 0; l < L; ++l) {
                    const double b = real_beta(st, tab, knew, a, j, l);
                    sum = l == 0 ? b : sum + b;
                }
                return sum;
            };
            for (int a = lane; a < n; a += 64) {
                double b = -INFINITY;
                if (a != i && (anynan || !(best32[a] < tau))) {
                    b = total(a, top[0]);
                    for (int c = 1; c < Mb; ++c) {
                        const double v = total(a, top[c]);
                        b = v > b ? v : b;
                    }
                }
                best[a] = b;
            }
            wave_sync();
            wave_topk<CAP, false>(best, n, N, topn, taken);
        }
    } else {  // profiling: valid placeholder competitors (agents 0..)
        for (int c = lane; c < N; c += 64) topn[c] = c;
        wave_sync();
    }
    // (d) competitor q's M/2 best tasks outside agent i's top M: the first M/2 entries of
    //     its topD list not in top[], stored ascending (largest picked first)
    const int mw = (m + 31) / 32;
    for (int w = lane; w < mw; w += 64) tmask[w] = 0u;
    wave_sync();
    for (int c = lane; c < M; c += 64) atomicOr(&tmask[top[c] >> 5], 1u << (top[c] & 31));
    wave_sync();
    auto in_top = [&](int j) { return ((tmask[j >> 5] >> (j & 31)) & 1u) != 0u; };
    for (int q = lane; q < N; q += 64) {
        const int *d = st.topD + (e * n + topn[q]) * (int64_t)MD;
        int got = 0;
        if (MD <= kObsMD) {  // the whole list in one round trip
            int dj[kObsMD];
#pragma unroll
            for (int c = 0; c < kObsMD; ++c) dj[c] = c < MD ? d[c] : 0;
#pragma unroll
            for (int c = 0; c < kObsMD; ++c) {
                if (c < MD && got < M2 && !in_top(dj[c])) {
                    oth[q * M2 + (M2 - 1 - got)] = dj[c];
                    ++got;
                }
            }
        } else {
            for (int c = 0; c < MD && got < M2; ++c) {
                const int j = d[c];
                if (!in_top(j)) oth[q * M2 + (M2 - 1 - got++)] = j;
            }
        }
    }
    wave_sync();
    // (e) the observation row: local, neighbouring, neighbouring-other benefits, assigns
    const int64_t o0 = foff(bv.obs, e, row, i, 0);
    const int r1 = M * L, r2 = r1 + N * M * L, r3 = r2 + N * M2 * L, r4 = r3 + M;
    const double *pw = st.power + e * n;
    // benefit entries are copied from the batch's beta row just written by the strip
    // kernel when it holds the same element type (the stored value is the same rounding
    // of the same float64: 3 L-contiguous elements per (agent, task) instead of 3 table
    // lines); otherwise recomputed from the table
    const bool copy = bv.beta.ptr && bv.beta.dtype == bv.obs.dtype;
    const int64_t b0 = copy ? foff(bv.beta, e, row, 0, 0) : 0;
    auto bval = [&](int a, int j, int l, int p) {
        if (copy) {
            const int64_t src = b0 + a * bv.beta.stride[2] + j * bv.beta.stride[3] + l;
            switch (bv.obs.dtype) {
                case ASG_F16:
                    reinterpret_cast<uint16_t *>(bv.obs.ptr)[o0 + p] = reinterpret_cast<const uint16_t *>(bv.beta.ptr)[src];
                    return;
                case ASG_F32:
                    reinterpret_cast<float *>(bv.obs.ptr)[o0 + p] = reinterpret_cast<const float *>(bv.beta.ptr)[src];
                    return;
                default:
                    reinterpret_cast<double *>(bv.obs.ptr)[o0 + p] = reinterpret_cast<const double *>(bv.beta.ptr)[src];
                    return;
            }
        }
        store_real(bv.obs, o0 + p, real_beta(st, tab, knew, a, j, l));
    };
    if (ASG_OBS_TWOPHASE && copy && bv.obs.dtype == ASG_F16 && osz <= 64 * kObsG && n < 65536 && m < 65536 &&
        !(ASG_REAL_PROF_SKIP & 16)) {
        // the row's benefit entries gathered from the beta row first, then stored: a load issued
        // behind a store waits for its acknowledgement (gfx9's in-order vmcnt).  Entry p is
        // element p % L of L-run p / L, whose (agent, task) the slot table holds
        const int nsl = M + N * M + N * M2;
        for (int sx = lane; sx < nsl; sx += 64) {
            int a, j;
            if (sx < M) {
                a = i, j = top[sx];
            } else if (sx < M + N * M) {
                const int x = sx - M, q = x / M;
                a = topn[q], j = top[x - q * M];
            } else {
                const int x = sx - M - N * M, q = x / M2;
                a = topn[q], j = oth[x];  // oth is [N][M2]: entry q * M2 + (x - q * M2) = x
            }
            slot[sx] = ((uint32_t)a << 16) | (uint32_t)j;
        }
        wave_sync();
        const uint16_t *bsrc = reinterpret_cast<const uint16_t *>(bv.beta.ptr) + b0;
        uint16_t *odst = reinterpret_cast<uint16_t *>(bv.obs.ptr) + o0;
        const int64_t bs2 = bv.beta.stride[2], bs3 = bv.beta.stride[3];
        const int sq = 64 / L, sr = 64 - sq * L;  // +64 entries = +sq runs, +sr elements
        uint32_t sv[kObsG];
        const int sl0 = lane / L, l0 = lane - sl0 * L;
        {
            int sl = sl0, l = l0;
#pragma unroll
            for (int g = 0; g < kObsG; ++g) {
                if (64 * g >= r3) break;
                sv[g] = lane + 64 * g < r3 ? slot[sl] : 0u;
                l += sr;
                sl += sq + (l >= L ? 1 : 0);
                l -= l >= L ? L : 0;
            }
        }
        uint16_t val[kObsG];
        {
            int l = l0;
#pragma unroll
            for (int g = 0; g < kObsG; ++g) {
                if (64 * g >= r3) break;
                const uint32_t t = sv[g];
                val[g] = lane + 64 * g < r3 ? bsrc[(int64_t)(t >> 16) * bs2 + (int64_t)(t & 0xffffu) * bs3 + l] : (uint16_t)0;
                l += sr;
                l -= l >= L ? L : 0;
            }
        }
#pragma unroll
        for (int g = 0; g < kObsG; ++g) {
            if (64 * g >= osz) break;
            const int p = lane + 64 * g;
            if (p < r3) {
                odst[p] = val[g];
            } else if (p < r4) {
                store_real(bv.obs, o0 + p, top[p - r3] == pi ? 1.0 : 0.0);
            } else if (p < osz) {  // [power_i, power[top_n]] (real_power_constellation_env.py:226-229)
                store_real(bv.obs, o0 + p, p == r4 ? pw[i] : pw[topn[p - r4 - 1]]);
            }
        }
        return;
    }
    for (int p = lane; p < ((ASG_REAL_PROF_SKIP & 16) ? 0 : osz); p += 64) {
        if (p < r1) {
            bval(i, top[p / L], p % L, p);
        } else if (p < r2) {
            const int x = p - r1, q = x / (M * L), y = x - q * M * L;
            bval(topn[q], top[y / L], y % L, p);
        } else if (p < r3) {
            const int x = p - r2, q = x / (M2 * L), y = x - q * M2 * L;
            bval(topn[q], oth[q * M2 + y / L], y % L, p);
        } else if (p < r4) {
            store_real(bv.obs, o0 + p, top[p - r3] == pi ? 1.0 : 0.0);
        } else {  // [power_i, power[top_n]] (real_power_constellation_env.py:226-229)
            store_real(bv.obs, o0 + p, p == r4 ? pw[i] : pw[topn[p - r4 - 1]]);
        }
    }
}

// host layout [E'][n][m][T] (the reference's sat_prox_mat) -> time-major [E'][T][n][m]
__global__ void real_table_transpose_kernel(const double *src, double *dst, int64_t count, int n, int m, int T) {
    const int64_t total = count * n * m * T;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = p / ((int64_t)T * n * m);
        int64_t r = p - e * (int64_t)T * n * m;
        const int k = (int)(r / ((int64_t)n * m));
        r -= (int64_t)k * n * m;
        const int i = (int)(r / m), j = (int)(r - (int64_t)i * m);
        dst[p] = src[((e * n + i) * m + j) * T + k];
    }
}

// ---- HAALSelector (action_selectors/non_rl_selectors.py:54-118) ---------------------------
// The reference forks (deepcopy) every env once per time-interval sequence of the lookahead
// window, and per interval solves scipy's LSA on beta_hat summed over L and steps the fork
// interval-length times.  A fork's state is (step, previous assignment, and in the power /
// interference variants the power states, drained or recharged by every step the fork takes:
// real_power_constellation_env.py:137-191): the benefits are the constant table.  Sequences
// share prefixes, so the distinct LSA states form a tree of decision nodes (decision time t,
// the assignment in force before it = the parent node's, the power replayed along the
// ancestors' steps): 2^(eff-1) nodes, solved level by level as batched LSAs over all envs,
// then every sequence's value is the reference's sum of per-step reward sums (each variant's
// own reward rule, real_step_rewards).
constexpr int kHaalMaxL = 6;                     // 2^(6-1) = 32 nodes / sequences
struct HaalPlan {
    int nodes, seqs, eff;
    int8_t node_t[1 << (kHaalMaxL - 1)];         // decision time offset of each node
    int8_t node_parent[1 << (kHaalMaxL - 1)];    // parent node or -1 (root: the env's prev)
    int8_t seq_len[1 << (kHaalMaxL - 1)];        // intervals per sequence
    int8_t seq_node[1 << (kHaalMaxL - 1)][kHaalMaxL];  // the decision node of each interval
};

// total beta_hat of one (node, env, agent) row: ((b0 - lambda * pen) + b1) + ... in numpy's
// order (real_constellation_env.py:309-326, then .sum(axis=-1) left to right).  Power variants
// (real_power_constellation_env.py:310-352, interference_constellation_env.py:355-406): the
// agent's power at the node's decision time, replayed from the env's along the ancestors'
// assignments; a row below 1e-12 power is all zeros; the interference variant's penalty mask is
// 1 - I whatever T_trans (interference_constellation_env.py:384).
__global__ void __launch_bounds__(256) haal_matrix_kernel(RealState st, int k, HaalPlan plan, int node0, int nodes,
                                                          const int64_t *assign, double *mats) {
    const int lane = threadIdx.x & 63;
    const int64_t gr = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // row over [nodes][E][n]
    const int n = st.n, m = st.m;
    if (gr >= (int64_t)nodes * st.E * n) return;
    const int i = (int)(gr % n);
    const int64_t ne = gr / n;
    const int64_t e = ne % st.E;
    const int node = node0 + (int)(ne / st.E);
    const int t = plan.node_t[node], par = plan.node_parent[node];
    const int prev = par < 0 ? st.prev[e * n + i] : (int)assign[((int64_t)par * st.E + e) * n + i];
    const double *tab = st.table + e * st.table_env_stride;
    double *row = mats + gr * m;
    bool poison = prev < 0 || prev >= m;
    bool dead = false;
    if (!poison && st.variant != ASG_REAL_PLAIN) {
        // the power this fork reaches at time t: the env's, then every step of the ancestors'
        // intervals (node chain root .. parent, each in force until its child's decision time)
        int chain[kHaalMaxL];
        int d = 0;
        for (int x = node; x >= 0 && d < kHaalMaxL; x = plan.node_parent[x]) chain[d++] = x;
        double p = st.power[e * n + i];
        for (int c = d - 1; c >= 1 && !poison; --c) {
            const int anc = chain[c];
            const int ai = (int)assign[((int64_t)anc * st.E + e) * n + i];
            if (ai < 0 || ai >= m) { poison = true; break; }
            for (int s2 = plan.node_t[anc]; s2 < plan.node_t[chain[c - 1]]; ++s2)
                if (p > 0) {  // real_power_update
                    if (real_beta(st, tab, k + s2, i, ai, 0) > 1e-12) {
                        p -= 0.2;
                    } else {
                        const double q = p + 0.1;
                        p = q < 1.0 ? q : 1.0;
                    }
                }
        }
        dead = p < 1e-12;  // np.where(sats_out_of_power, 0, beta_hat)
    }
    if (poison) {
        // the parent node's LSA failed (its assignment is -1 rows): poison this row so the
        // node's LSA reports invalid entries too, never index T_trans with it
        for (int j = lane; j < m; j += 64) row[j] = __builtin_nan("");
        return;
    }
    if (dead) {
        for (int j = lane; j < m; j += 64) row[j] = 0.0;
        return;
    }
    const bool eye = st.variant == ASG_REAL_INTERFERENCE;
    for (int j = lane; j < m; j += 64) {
        double s = real_beta(st, tab, k + t, i, j, 0);
        const double b0 = s;
        for (int l = 1; l < st.L; ++l) s = s + real_beta(st, tab, k + t, i, j, l);
        const double cond = s > 1e-12 ? 1.0 : 0.0;
        const double pen = (eye ? (prev != j ? 1.0 : 0.0) : st.T_trans[(int64_t)prev * m + j]) * cond;
        double tot = b0 - st.lambda_ * pen;
        for (int l = 1; l < st.L; ++l) tot = tot + real_beta(st, tab, k + t, i, j, l);
        row[j] = tot;
    }
}

// value of every (env, sequence): sum over its steps of Python's sum(rewards) (agent order,
// float64), one workgroup per (sequence, env), each step by the variant's own reward rule and,
// in the power variants, the fork's power carried from step to step; then (a second launch)
// the best sequence per env
__host__ __device__ __forceinline__ size_t haal_values_lds(int n, int m) {
    return (size_t)16 * n + (size_t)4 * (3 * n + m) + 16;  // rewards, power | tasks, prev, applicable, counts, flag
}

__global__ void __launch_bounds__(256) haal_values_kernel(RealState st, int k, HaalPlan plan, const int64_t *assign,
                                                          double *values) {
    extern __shared__ double s_rew[];  // [n] rewards, [n] power, then ints: [n] tasks, [n] prev, [n] applicable, [m] counts
    const int n = st.n, m = st.m;
    double *spw = s_rew + n;
    int *sa = reinterpret_cast<int *>(spw + n);
    int *sp = sa + n, *sapp = sp + n, *scnt = sapp + n;
    int *sbad = scnt + m;
    const int s = blockIdx.x % plan.seqs;
    const int64_t e = blockIdx.x / plan.seqs;
    const double *tab = st.table + e * st.table_env_stride;
    for (int i = threadIdx.x; i < n; i += blockDim.x) spw[i] = st.variant != ASG_REAL_PLAIN ? st.power[e * n + i] : 1.0;
    double tot = 0.0;
    bool bad = false;
    for (int iv = 0; iv < plan.seq_len[s] && !bad; ++iv) {
        const int node = plan.seq_node[s][iv];
        const int t0 = plan.node_t[node];
        const int t1 = iv + 1 < plan.seq_len[s] ? plan.node_t[plan.seq_node[s][iv + 1]] - 1 : plan.eff - 1;
        const int64_t *A = assign + ((int64_t)node * st.E + e) * n;
        const int par = plan.node_parent[node];
        for (int t = t0; t <= t1; ++t) {
            if (threadIdx.x == 0) *sbad = 0;
            __syncthreads();
            for (int i = threadIdx.x; i < n; i += blockDim.x) {
                // the previous assignment: the parent's on the interval's first step, then A
                const int p = t > t0 ? (int)A[i]
                                     : (par < 0 ? st.prev[e * n + i] : (int)assign[((int64_t)par * st.E + e) * n + i]);
                const int c = (int)A[i];
                sa[i] = c;
                sp[i] = p;
                if (c < 0 || c >= m || p < 0 || p >= m) *sbad = 1;
            }
            __syncthreads();
            if (*sbad) {
                // a failed LSA upstream (-1 assignment rows): the sequence's value is NaN and
                // the env's status carries the LSA error
                bad = true;
                break;
            }
            real_step_rewards(st, tab, k + t, sa, [&](int i) { return sp[i]; }, spw, scnt, sapp, s_rew);
            __syncthreads();
            if (threadIdx.x == 0) {
                double r = 0.0;
                for (int i = 0; i < n; ++i) r += s_rew[i];  // sum(rewards), left to right
                tot += r;                                   // total_tis_value += sum(rewards)
            }
            if (st.variant != ASG_REAL_PLAIN) real_power_update(st, tab, k + t, sa, spw);
            __syncthreads();
        }
    }
    if (threadIdx.x == 0) values[e * plan.seqs + s] = bad ? __builtin_nan("") : tot;
}

// per env: the first sequence with the largest value (strict >), its first-interval
// assignment (the root node's: every sequence starts at the fork state) as float task ids
__global__ void haal_pick_kernel(int64_t E, int n, int seqs, const double *values, const int64_t *assign,
                                 const int32_t *lsa_status, float *col_out, int32_t *best_out, int32_t *status_out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    double best = -INFINITY;
    int bs = -1;
    for (int s = 0; s < seqs; ++s) {
        const double v = values[e * seqs + s];
        if (v > best) {
            best = v;
            bs = s;
        }
    }
    if (best_out) best_out[e] = bs;
    int32_t st = lsa_status ? lsa_status[e] : 0;
    if (st == 0 && bs < 0) st = ASG_E_INVALID_ARG;  // every value NaN: the reference's best_assignment is None
    if (status_out) status_out[e] = st;
    for (int i = 0; i < n; ++i) col_out[e * n + i] = (st == 0) ? (float)assign[e * n + i] : -1.0f;
}

// min over the levels' LSA status words of each env ([levels' B] -> [E])
__global__ void haal_status_kernel(const int32_t *st_all, int64_t rows, int64_t E, int32_t *st_env) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    int32_t v = 0;
    for (int64_t r = e; r < rows; r += E) v = st_all[r] < v ? st_all[r] : v;
    st_env[e] = v;
}

}  // namespace asg

using asg::RealState;

struct asg_real_handle {
    RealState st{};
    hipStream_t stream = nullptr;
    int device = 0;
    int k = 0;
    bool has_reset = false;
    bool table_ready = false;
    double *table_buf = nullptr;
    void *haal_ws = nullptr;  // HAAL workspace (grown on demand)
    size_t haal_ws_bytes = 0;
    int64_t *bids_assign = nullptr;   // bids_as_actions: [E][n] assignments of the step's LSA
    int32_t *bids_status = nullptr;   // [E] its status
    std::string err;
};

namespace {

int rfail(asg_real_handle *h, int code, const std::string &msg) {
    asg::set_last_error(msg);
    if (h) h->err = msg;
    return code;
}
int rhip(asg_real_handle *h, hipError_t e, const char *what) {
    return rfail(h, ASG_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct RDeviceGuard {
    int prev = -1;
    explicit RDeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~RDeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

bool rfield_ok(const asg_field &f, std::initializer_list<int> ok) {
    if (!f.ptr) return true;
    for (int d : ok)
        if (f.dtype == d) return true;
    return false;
}

int rcheck_view(asg_real_handle *h, const asg_batch_view *b, bool step) {
    if (!b) return rfail(h, ASG_E_INVALID_ARG, "batch view is NULL");
    if (!b->obs.ptr) return rfail(h, ASG_E_INVALID_ARG, "obs field is required");
    const bool ok = rfield_ok(b->obs, {ASG_F16, ASG_F32, ASG_F64}) && rfield_ok(b->beta, {ASG_F16, ASG_F32, ASG_F64}) &&
                    rfield_ok(b->rewards, {ASG_F16, ASG_F32, ASG_F64}) && rfield_ok(b->avail_actions, {ASG_BOOL}) &&
                    rfield_ok(b->terminated, {ASG_BOOL}) &&
                    rfield_ok(b->prev_assigns, {ASG_I16, ASG_I32, ASG_I64}) &&
                    rfield_ok(b->actions_onehot, {ASG_I16, ASG_I32, ASG_I64}) && rfield_ok(b->filled, {ASG_I64});
    if (!ok) return rfail(h, ASG_E_INVALID_ARG, "batch field dtype does not match the real-env scheme");
    if (step && h->st.bids && (!b->actions.ptr || !rfield_ok(b->actions, {ASG_F32})))
        return rfail(h, ASG_E_INVALID_ARG, "bids_as_actions expects float32 actions [B, T+1, n, m]");
    if (step && !h->st.bids && (!b->actions.ptr || !rfield_ok(b->actions, {ASG_I16, ASG_I32, ASG_I64})))
        return rfail(h, ASG_E_INVALID_ARG, "step needs integer actions");
    return ASG_OK;
}

// candidates per lane of a top-K over `len` values: 1, 2, 4, 6, 8, 16, or 0 (> 1024: rescans);
// 6 (257..384, e.g. the 324 satellites) sorts its lanes with a 12-comparator network
int cap_of(int len) {
    const int c = (len + 63) / 64;
    return c <= 1 ? 1 : c <= 2 ? 2 : c <= 4 ? 4 : c <= 6 ? 6 : c <= 8 ? 8 : c <= 16 ? 16 : 0;
}

int strip_height(const RealState &st) {
    int S = 16;
    while (S > 1 && asg::strip_lds(S, st.m) > 64 * 1024) S >>= 1;
    return S;
}

// reset: reset + strip + observation passes; step: transition, strip, observation
hipError_t launch_real(asg_real_handle *h, const asg_real_batch_view &v, int ts, bool step) {
    const RealState &st = h->st;
    const asg_batch_view &bv = v.base;
    const int knew = step ? h->k + 1 : 0;
    const int row = step ? ts + 1 : ts;
    if (step) {
        RealState tst = st;
        if (st.bids) {
            // the step's LSA(bids row ts, maximize) for every env in one batched launch (the
            // scipy-exact solver, rectangular n <= m, float32 bids read in place; asg_lsa.hip)
            const float *row0 = static_cast<const float *>(bv.actions.ptr) + (int64_t)ts * bv.actions.stride[1];
            const int64_t str[3] = {bv.actions.stride[0], bv.actions.stride[2], bv.actions.stride[3]};
            hipError_t e0 = asg::launch_lsa_batched(row0, ASG_F32, str, st.E, st.n, st.m, 1, nullptr, h->bids_assign,
                                                    h->bids_status, h->stream);
            if (e0 != hipSuccess) return e0;
            tst.assign = h->bids_assign;
            tst.assign_status = h->bids_status;
        }
        hipLaunchKernelGGL(asg::real_transition_kernel, dim3((unsigned)st.E), dim3(256), asg::transition_lds(st.n, st.m),
                           h->stream, bv, tst, ts, h->k);
    } else {
        hipLaunchKernelGGL(asg::real_reset_kernel, dim3((unsigned)st.E), dim3(256), sizeof(int) * (size_t)st.m,
                           h->stream, st);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int S = strip_height(st);
    const dim3 sgrid((unsigned)((st.n + S - 1) / S), (unsigned)st.E);
    const size_t slds = asg::strip_lds(S, st.m);
#define STRIP_(CAP) \
    hipLaunchKernelGGL(asg::real_strip_kernel<CAP>, sgrid, dim3(64 * S), slds, h->stream, bv, v.power_states, st, ts, \
                       knew, (int)step, S)
    switch (cap_of(st.m)) {
        case 1: STRIP_(1); break;
        case 2: STRIP_(2); break;
        case 4: STRIP_(4); break;
        case 8: STRIP_(8); break;
        case 6: STRIP_(6); break;
        case 16: STRIP_(16); break;
        default: STRIP_(0); break;
    }
#undef STRIP_
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t per_wave = asg::real_obs_lds_per_wave(st.n, st.m, st.N, st.M);
    int waves = 4;
    while (waves > 1 && per_wave * waves > 64 * 1024) waves >>= 1;
    const int G = (st.n + waves - 1) / waves;
    const dim3 grid((unsigned)(8 * ((st.E + 7) / 8) * G));
#define OBS_(CAP)                                                                                                 \
    hipLaunchKernelGGL(asg::real_obs_kernel<CAP>, grid, dim3(64 * waves), per_wave * waves, h->stream, bv, st, row, \
                       knew, G)
    switch (cap_of(st.n)) {
        case 1: OBS_(1); break;
        case 2: OBS_(2); break;
        case 4: OBS_(4); break;
        case 8: OBS_(8); break;
        case 6: OBS_(6); break;
        case 16: OBS_(16); break;
        default: OBS_(0); break;
    }
#undef OBS_
    return hipGetLastError();
}

template <class T>
hipError_t upload(T **dst, const T *src, size_t count) {
    hipError_t e = hipMalloc(dst, sizeof(T) * count);
    if (e == hipSuccess) e = hipMemcpy(*dst, src, sizeof(T) * count, hipMemcpyHostToDevice);
    return e;
}

}  // namespace

extern "C" {

int asg_real_create(const asg_real_config *cfg, int device, void *hip_stream, asg_real_handle **out) {
    if (!cfg || !out) return rfail(nullptr, ASG_E_INVALID_ARG, "NULL config or output");
    *out = nullptr;
    const int n = cfg->n, m = cfg->m, T = cfg->T;
    const int L = cfg->L < T ? cfg->L : T;  // self.L = min(L, T) (:37)
    if (cfg->num_envs <= 0 || n <= 0 || m <= 0 || T <= 0 || cfg->L <= 0)
        return rfail(nullptr, ASG_E_INVALID_ARG, "num_envs, n, m, T, L must be positive");
    if (cfg->variant < ASG_REAL_PLAIN || cfg->variant > ASG_REAL_INTERFERENCE)
        return rfail(nullptr, ASG_E_INVALID_ARG, "unknown variant");
    if (n > m)
        return rfail(nullptr, ASG_E_INVALID_ARG,
                     "Cannot take a larger sample than population when 'replace=False' (prev_assigns needs n <= m)");
    if (n > 4096 || m > 4096) return rfail(nullptr, ASG_E_INVALID_ARG, "n, m <= 4096");
    if (cfg->M <= 0 || cfg->M > m || cfg->M % 2 != 0)
        return rfail(nullptr, ASG_E_INVALID_ARG, "M must be even and in [2, m] (obs size uses N*M//2)");
    if (cfg->N <= 0 || cfg->N > n) return rfail(nullptr, ASG_E_INVALID_ARG, "N must be in [1, n]");
    if (m < cfg->M + cfg->M / 2)
        return rfail(nullptr, ASG_E_INVALID_ARG, "m must be >= M + M/2 (the competitors' other tasks)");
    if (asg::real_obs_lds_per_wave(n, m, cfg->N, cfg->M) > 64 * 1024 || asg::strip_lds(1, m) > 64 * 1024)
        return rfail(nullptr, ASG_E_INVALID_ARG, "n, m, N, M too large for the observation kernels");
    if (cfg->variant == ASG_REAL_INTERFERENCE && (!cfg->sat_freq_bands || !cfg->neighbor_matrix))
        return rfail(nullptr, ASG_E_INVALID_ARG, "the interference variant needs sat_freq_bands and neighbor_matrix");
    RDeviceGuard g(device);
    auto *h = new (std::nothrow) asg_real_handle();
    if (!h) return rfail(nullptr, ASG_E_INVALID_ARG, "out of host memory");
    h->device = device;
    h->stream = static_cast<hipStream_t>(hip_stream);
    RealState &st = h->st;
    st.E = cfg->num_envs;
    st.n = n, st.m = m, st.T = T, st.L = L, st.N = cfg->N, st.M = cfg->M;
    st.lambda_ = cfg->lambda_;
    st.variant = cfg->variant;
    st.seed = cfg->seed;
    st.env_base = cfg->env_index_base;
    st.bids = cfg->bids_as_actions ? 1 : 0;
    std::vector<double> hp(m, 1.0), ht((size_t)m * m), hn((size_t)m * m, 0.0);
    std::vector<int> hb(n, 0);
    if (cfg->task_prios) std::memcpy(hp.data(), cfg->task_prios, sizeof(double) * m);
    for (int a = 0; a < m; ++a)
        for (int b = 0; b < m; ++b) ht[(size_t)a * m + b] = cfg->T_trans ? cfg->T_trans[(size_t)a * m + b] : (a != b);
    if (cfg->neighbor_matrix) std::memcpy(hn.data(), cfg->neighbor_matrix, sizeof(double) * (size_t)m * m);
    if (cfg->sat_freq_bands) std::memcpy(hb.data(), cfg->sat_freq_bands, sizeof(int) * n);
    double *prios = nullptr, *tt = nullptr, *nb = nullptr;
    int *bands = nullptr;
    hipError_t e = upload(&prios, hp.data(), hp.size());
    if (e == hipSuccess) e = upload(&tt, ht.data(), ht.size());
    if (e == hipSuccess) e = upload(&nb, hn.data(), hn.size());
    if (e == hipSuccess) e = upload(&bands, hb.data(), hb.size());
    st.prios = prios, st.T_trans = tt, st.nbr = nb, st.bands = bands;
    if (e == hipSuccess) e = hipMalloc(&st.prev, sizeof(int) * (size_t)st.E * n);
    if (e == hipSuccess) e = hipMalloc(&st.power, sizeof(double) * (size_t)st.E * n);
    if (e == hipSuccess) e = hipMalloc(&st.returns, sizeof(double) * (size_t)st.E);
    if (e == hipSuccess) e = hipMalloc(&st.totT, sizeof(float) * (size_t)st.E * n * m);
    if (e == hipSuccess) e = hipMalloc(&st.topA, sizeof(int) * (size_t)st.E * n * cfg->M);
    if (e == hipSuccess) e = hipMalloc(&st.topD, sizeof(int) * (size_t)st.E * n * (cfg->M + cfg->M / 2));
    if (e == hipSuccess) e = hipMalloc(&st.err, sizeof(int));
    if (e == hipSuccess) e = hipMemset(st.err, 0, sizeof(int));
    if (e == hipSuccess) e = hipMemset(st.returns, 0, sizeof(double) * (size_t)st.E);
    if (e == hipSuccess && st.bids) e = hipMalloc(&h->bids_assign, sizeof(int64_t) * (size_t)st.E * n);
    if (e == hipSuccess && st.bids) e = hipMalloc(&h->bids_status, sizeof(int32_t) * (size_t)st.E);
    if (e != hipSuccess) {
        asg_real_destroy(h);
        return rhip(nullptr, e, "asg_real_create");
    }
    *out = h;
    return ASG_OK;
}

void asg_real_destroy(asg_real_handle *h) {
    if (!h) return;
    RDeviceGuard g(h->device);
    hipFree(const_cast<double *>(h->st.prios));
    hipFree(const_cast<double *>(h->st.T_trans));
    hipFree(const_cast<double *>(h->st.nbr));
    hipFree(const_cast<int *>(h->st.bands));
    hipFree(const_cast<int64_t *>(h->st.prev0));
    hipFree(h->st.prev);
    hipFree(h->st.power);
    hipFree(h->st.returns);
    hipFree(h->st.totT);
    hipFree(h->st.topA);
    hipFree(h->st.topD);
    hipFree(h->st.err);
    hipFree(h->table_buf);
    hipFree(h->haal_ws);
    hipFree(h->bids_assign);
    hipFree(h->bids_status);
    delete h;
}

int asg_real_set_initial_assignments(asg_real_handle *h, const int64_t *prev0, int64_t count, int on_device) {
    if (!h) return rfail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    RDeviceGuard g(h->device);
    hipFree(const_cast<int64_t *>(h->st.prev0));
    h->st.prev0 = nullptr;
    if (!prev0) return ASG_OK;  // back to Philox draws
    if (count != 1 && count != h->st.E) return rfail(h, ASG_E_INVALID_ARG, "count must be 1 or num_envs");
    const size_t elems = (size_t)count * h->st.n;
    std::vector<int64_t> host(elems);
    hipError_t e = hipSuccess;
    if (on_device) {
        e = hipMemcpyAsync(host.data(), prev0, sizeof(int64_t) * elems, hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    } else {
        std::memcpy(host.data(), prev0, sizeof(int64_t) * elems);
    }
    if (e != hipSuccess) return rhip(h, e, "asg_real_set_initial_assignments");
    for (size_t c = 0; c < (size_t)count; ++c) {  // choice(m, n, replace=False): distinct tasks in [0, m)
        std::vector<char> seen(h->st.m, 0);
        for (int i = 0; i < h->st.n; ++i) {
            const int64_t v = host[c * h->st.n + i];
            if (v < 0 || v >= h->st.m || seen[v])
                return rfail(h, ASG_E_INVALID_ARG, "initial assignments must be distinct tasks in [0, m)");
            seen[v] = 1;
        }
    }
    int64_t *dev = nullptr;
    e = upload(&dev, host.data(), elems);
    if (e != hipSuccess) return rhip(h, e, "asg_real_set_initial_assignments");
    h->st.prev0 = dev;
    h->st.prev0_env_stride = count == 1 ? 0 : h->st.n;
    return ASG_OK;
}

int asg_real_set_benefits(asg_real_handle *h, const double *table, int64_t count, int on_device) {
    if (!h || !table) return rfail(h, ASG_E_INVALID_ARG, "NULL handle or table");
    if (count != 1 && count != h->st.E) return rfail(h, ASG_E_INVALID_ARG, "count must be 1 or num_envs");
    RDeviceGuard g(h->device);
    const RealState &st = h->st;
    const size_t elems = (size_t)count * st.n * st.m * st.T;
    hipFree(h->table_buf);
    h->table_buf = nullptr;
    double *src = nullptr;
    hipError_t e = hipMalloc(&h->table_buf, sizeof(double) * elems);
    if (e == hipSuccess && !on_device) {
        e = hipMalloc(&src, sizeof(double) * elems);
        if (e == hipSuccess) e = hipMemcpyAsync(src, table, sizeof(double) * elems, hipMemcpyHostToDevice, h->stream);
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(asg::real_table_transpose_kernel, dim3(2048), dim3(256), 0, h->stream,
                           on_device ? table : src, h->table_buf, (int64_t)count, st.n, st.m, st.T);
        e = hipGetLastError();
    }
    if (src) {
        const hipError_t e2 = hipStreamSynchronize(h->stream);
        hipFree(src);
        if (e == hipSuccess) e = e2;
    }
    if (e != hipSuccess) return rhip(h, e, "asg_real_set_benefits");
    h->st.table = h->table_buf;
    h->st.table_env_stride = count == 1 ? 0 : (int64_t)st.T * st.n * st.m;
    h->table_ready = true;
    return ASG_OK;
}

int asg_real_set_stream(asg_real_handle *h, void *hip_stream) {
    if (!h) return rfail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    h->stream = static_cast<hipStream_t>(hip_stream);
    return ASG_OK;
}

int asg_real_reset(asg_real_handle *h, const asg_real_batch_view *view, int ts) {
    if (!h) return rfail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    if (!h->table_ready) return rfail(h, ASG_E_STATE, "asg_real_reset: no benefit table (asg_real_set_benefits)");
    if (!view) return rfail(h, ASG_E_INVALID_ARG, "batch view is NULL");
    if (int rc = rcheck_view(h, &view->base, false)) return rc;
    if (view->power_states.ptr && !rfield_ok(view->power_states, {ASG_F16, ASG_F32, ASG_F64}))
        return rfail(h, ASG_E_INVALID_ARG, "power_states must be a float field");
    RDeviceGuard g(h->device);
    if (h->has_reset) h->st.episode += 1;  // Philox counter: a fresh draw every episode
    const hipError_t e = launch_real(h, *view, ts, false);
    if (e != hipSuccess) return rhip(h, e, "asg_real_reset");
    h->k = 0;
    h->has_reset = true;
    return ASG_OK;
}

int asg_real_step(asg_real_handle *h, const asg_real_batch_view *view, int ts) {
    if (!h) return rfail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    if (!h->has_reset) return rfail(h, ASG_E_STATE, "asg_real_step before asg_real_reset");
    if (h->k >= h->st.T) return rfail(h, ASG_E_STATE, "episode is done: call asg_real_reset");
    if (!view) return rfail(h, ASG_E_INVALID_ARG, "batch view is NULL");
    if (int rc = rcheck_view(h, &view->base, true)) return rc;
    if (view->power_states.ptr && !rfield_ok(view->power_states, {ASG_F16, ASG_F32, ASG_F64}))
        return rfail(h, ASG_E_INVALID_ARG, "power_states must be a float field");
    RDeviceGuard g(h->device);
    const hipError_t e = launch_real(h, *view, ts, true);
    if (e != hipSuccess) return rhip(h, e, "asg_real_step");
    h->k += 1;
    return ASG_OK;
}

int asg_real_sync_status(asg_real_handle *h) {
    if (!h) return rfail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    RDeviceGuard g(h->device);
    int code = 0;
    hipError_t e = hipMemcpyAsync(&code, h->st.err, sizeof(int), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return rhip(h, e, "asg_real_sync_status");
    if (code != 0) (void)hipMemsetAsync(h->st.err, 0, sizeof(int), h->stream);
    if (code == ASG_E_ACTION_RANGE) return rfail(h, code, "action out of range [0, m)");
    if (code == ASG_E_LSA_INVALID) return rfail(h, code, "matrix contains invalid numeric entries");
    if (code == ASG_E_LSA_INFEASIBLE) return rfail(h, code, "cost matrix is infeasible");
    return code ? rfail(h, code, "device error") : ASG_OK;
}

int asg_real_get_returns(asg_real_handle *h, double *out_device) {
    if (!h || !out_device) return rfail(h, ASG_E_INVALID_ARG, "NULL handle or output");
    RDeviceGuard g(h->device);
    const hipError_t e = hipMemcpyAsync(out_device, h->st.returns, sizeof(double) * (size_t)h->st.E,
                                        hipMemcpyDeviceToDevice, h->stream);
    return e == hipSuccess ? ASG_OK : rhip(h, e, "asg_real_get_returns");
}

int asg_real_get_step(const asg_real_handle *h, int *k_out) {
    if (!h || !k_out) return rfail(nullptr, ASG_E_INVALID_ARG, "NULL handle or output");
    *k_out = h->k;
    return ASG_OK;
}

int asg_real_obs_size(int N, int M, int L) { return M * L + N * M * L + ((N * M) / 2) * L + M; }

// the decision tree and sequence list of HAALSelector's window (utils/methods.py:309-349:
// sequences depth first, the shorter first interval first)
static void haal_plan(int eff, asg::HaalPlan &p) {
    std::vector<std::vector<int>> seqs;  // decision times of each sequence
    std::vector<int> cur;
    std::function<void(int)> rec = [&](int last) {
        if (last == eff - 1) {
            seqs.push_back(cur);
            return;
        }
        for (int j = last + 1; j < eff; ++j) {
            cur.push_back(last + 1);
            rec(j);
            cur.pop_back();
        }
    };
    rec(-1);
    // nodes = distinct decision-time prefixes, numbered level by level
    std::vector<std::vector<int>> nodes;
    for (int lev = 1; lev <= eff; ++lev)
        for (const auto &sq : seqs)
            if ((int)sq.size() >= lev) {
                std::vector<int> pre(sq.begin(), sq.begin() + lev);
                if (std::find(nodes.begin(), nodes.end(), pre) == nodes.end()) nodes.push_back(pre);
            }
    p.eff = eff;
    p.nodes = (int)nodes.size();
    p.seqs = (int)seqs.size();
    for (int a = 0; a < p.nodes; ++a) {
        p.node_t[a] = (int8_t)nodes[a].back();
        std::vector<int> par(nodes[a].begin(), nodes[a].end() - 1);
        p.node_parent[a] = (int8_t)(par.empty() ? -1 : std::find(nodes.begin(), nodes.end(), par) - nodes.begin());
    }
    for (int s = 0; s < p.seqs; ++s) {
        p.seq_len[s] = (int8_t)seqs[s].size();
        for (size_t j = 0; j < seqs[s].size(); ++j) {
            std::vector<int> pre(seqs[s].begin(), seqs[s].begin() + j + 1);
            p.seq_node[s][j] = (int8_t)(std::find(nodes.begin(), nodes.end(), pre) - nodes.begin());
        }
    }
}

int asg_real_haal_num_sequences(const asg_real_handle *h) {
    if (!h) return rfail(nullptr, ASG_E_INVALID_ARG, "NULL handle");
    const int eff = std::min(h->st.L, h->st.T - h->k);
    return eff > 0 ? 1 << (eff - 1) : 0;
}

int asg_real_haal_select(asg_real_handle *h, float *col_out, double *values_out, int32_t *best_out,
                         int32_t *status_out) {
    if (!h || !col_out) return rfail(h, ASG_E_INVALID_ARG, "NULL handle or output");
    if (!h->has_reset) return rfail(h, ASG_E_STATE, "asg_real_haal_select before asg_real_reset");
    const asg::RealState &st = h->st;
    const int eff = std::min(st.L, st.T - h->k);
    if (eff <= 0) return rfail(h, ASG_E_STATE, "asg_real_haal_select: the episode is done");
    if (eff > asg::kHaalMaxL) return rfail(h, ASG_E_INVALID_ARG, "asg_real_haal_select: lookahead window > 6");
    asg::HaalPlan plan{};
    haal_plan(eff, plan);
    RDeviceGuard g(h->device);
    const int n = st.n, m = st.m;
    const int64_t E = st.E;
    int max_level = 0;  // nodes per level: level = prefix length
    {
        std::vector<int> per(eff + 1, 0);
        for (int a = 0; a < plan.nodes; ++a) {
            int d = 0;
            for (int x = a; x >= 0; x = plan.node_parent[x]) ++d;
            ++per[d];
        }
        for (int d = 1; d <= eff; ++d) max_level = std::max(max_level, per[d]);
    }
    // workspace: matrices of the largest level, all nodes' assignments, values, LSA status
    const size_t mats_b = sizeof(double) * (size_t)max_level * E * n * m;
    const size_t asg_b = sizeof(int64_t) * (size_t)plan.nodes * E * n;
    const size_t val_b = sizeof(double) * (size_t)E * plan.seqs;
    const size_t st_b = sizeof(int32_t) * (size_t)plan.nodes * E;
    const size_t need = mats_b + asg_b + val_b + st_b + 4 * 256;
    hipError_t e = hipSuccess;
    if (h->haal_ws_bytes < need) {
        e = hipStreamSynchronize(h->stream);
        hipFree(h->haal_ws);
        h->haal_ws = nullptr;
        h->haal_ws_bytes = 0;
        if (e == hipSuccess) e = hipMalloc(&h->haal_ws, need);
        if (e != hipSuccess) return rhip(h, e, "asg_real_haal_select (workspace)");
        h->haal_ws_bytes = need;
    }
    auto align = [](size_t x) { return (x + 255) & ~(size_t)255; };
    char *base = static_cast<char *>(h->haal_ws);
    double *mats = reinterpret_cast<double *>(base);
    int64_t *assign = reinterpret_cast<int64_t *>(base + align(mats_b));
    double *values = reinterpret_cast<double *>(base + align(mats_b) + align(asg_b));
    int32_t *lsa_st = reinterpret_cast<int32_t *>(base + align(mats_b) + align(asg_b) + align(val_b));
    // nodes are numbered level by level: [node0, node0 + cnt) is one level
    int node0 = 0;
    while (node0 < plan.nodes && e == hipSuccess) {
        int d0 = 0;
        for (int x = node0; x >= 0; x = plan.node_parent[x]) ++d0;
        int cnt = 0;
        while (node0 + cnt < plan.nodes) {
            int d = 0;
            for (int x = node0 + cnt; x >= 0; x = plan.node_parent[x]) ++d;
            if (d != d0) break;
            ++cnt;
        }
        const int64_t rows = (int64_t)cnt * E * n;
        hipLaunchKernelGGL(asg::haal_matrix_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, h->stream, st,
                           h->k, plan, node0, cnt, assign, mats);
        e = hipGetLastError();
        if (e == hipSuccess) {
            const int64_t strides[3] = {(int64_t)n * m, m, 1};
            e = asg::launch_lsa_batched(mats, ASG_F64, strides, (int64_t)cnt * E, n, m, 1, nullptr,
                                        assign + (int64_t)node0 * E * n, lsa_st + (int64_t)node0 * E, h->stream);
        }
        node0 += cnt;
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(asg::haal_values_kernel, dim3((unsigned)(E * plan.seqs)), dim3(256),
                           asg::haal_values_lds(n, m), h->stream, st, h->k, plan, assign, values);
        e = hipGetLastError();
    }
    int32_t *st_env = lsa_st;  // reduced in place into the first E words (row e is env e of level 0)
    if (e == hipSuccess) {
        hipLaunchKernelGGL(asg::haal_status_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, h->stream, lsa_st,
                           (int64_t)plan.nodes * E, E, st_env);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(asg::haal_pick_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, h->stream, E, n,
                           plan.seqs, values, assign, st_env, col_out, best_out, status_out);
        e = hipGetLastError();
    }
    if (e == hipSuccess && values_out)
        e = hipMemcpyAsync(values_out, values, val_b, hipMemcpyDeviceToDevice, h->stream);
    return e == hipSuccess ? ASG_OK : rhip(h, e, "asg_real_haal_select");
}

}  // extern "C"

