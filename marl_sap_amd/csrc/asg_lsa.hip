// asg_lsa.hip -- batched scipy-exact linear sum assignment, beta_hat and the fused HAA
// selector (gfx950).  One wave64 per problem; the working cost matrix sits in LDS when
// it fits (48 KiB budget per wave), otherwise it is read in place from global memory
// (L2-resident for the row sweeps).
// Reference call sites: sap_selectors.py:32,90 (SAP selectors on Q-values),
// non_rl_selectors.py:36-47 (HAA: beta_hat + LSA), mock_constellation_env.py:228-274.
#include <stdlib.h>

#include <type_traits>

#include "asg_device.h"
#include "asg_internal.h"
#include "lsa_wave.h"
#include "sap_stage.h"

namespace asg {

constexpr size_t kLdsCostBudget = 48 * 1024;


// working matrix read in place: transposed when nr0 > nc0, negated for maximize
template <typename IT>
struct GlobalCost {
    static constexpr bool kInMemory = true;
    const IT *C;
    int64_t rs, cs;
    bool tr, neg;
    __device__ double operator()(int i, int j) const {
        const double x = (double)(tr ? C[(int64_t)j * rs + (int64_t)i * cs] : C[(int64_t)i * rs + (int64_t)j * cs]);
        return neg ? -x : x;
    }
};

template <typename IT>
__device__ int lsa_check_wave(const IT *C, int64_t rs, int64_t cs, int nr0, int nc0, bool maximize) {
    const int lane = threadIdx.x & (kWave - 1);
    int bad = 0;
    for (int idx = lane; idx < nr0 * nc0; idx += kWave) {
        const int r = idx / nc0, c = idx - r * nc0;
        double x = (double)C[r * rs + c * cs];
        if (maximize) x = -x;
        bad |= (x != x) || (x == -__builtin_inf());
    }
    return wave_or_i32(bad) ? ASG_E_LSA_INVALID : ASG_OK;
}

// Solve with the smallest columns-per-lane that fits, then hand the register-resident
// assignment to `emit(col4row)` (a generic lambda taking int (&)[CPL]).
template <int CPL, class Acc, class Emit>
__device__ int solve_emit_cpl(const Acc &acc, int nr, int nc, Emit &emit) {
    int c4r[CPL];
    const int status = lsa_solve_wave<CPL>(acc, nr, nc, c4r);
    if (status == ASG_OK) emit(c4r);
    return status;
}

// columns per lane for a working matrix of nc columns (one kernel instantiation each,
// so the register budget of a 64-column problem is not that of a 1024-column one)
static int cpl_for(int nc) { return nc <= 64 ? 1 : nc <= 128 ? 2 : nc <= 256 ? 4 : nc <= 512 ? 8 : 16; }

#define ASG_DISPATCH_CPL(nc, LAUNCH) \
    switch (cpl_for(nc)) {            \
        case 1: LAUNCH(1); break;     \
        case 2: LAUNCH(2); break;     \
        case 4: LAUNCH(4); break;     \
        case 8: LAUNCH(8); break;     \
        default: LAUNCH(16); break;   \
    }

// LDS carve: [cost (optional)][mark: nr0 ints]
template <int CPL, typename IT, typename CT, bool LDS_COST>
__global__ void __launch_bounds__(64) lsa_batched_kernel(const IT *C, int64_t s0, int64_t s1, int64_t s2, int nr0,
                                                         int nc0, int maximize, int64_t *row_out, int64_t *col_out,
                                                         int32_t *status_out) {
    extern __shared__ double s_lsa[];
    const int64_t b = blockIdx.x;
    const IT *Cb = C + b * s0;
    const bool tr = nc0 < nr0;
    const int nr = tr ? nc0 : nr0, nc = tr ? nr0 : nc0;
    const int k = nr;
    char *p = reinterpret_cast<char *>(s_lsa);
    CT *cost = reinterpret_cast<CT *>(p);
    if (LDS_COST) p += ((sizeof(CT) * (size_t)nr * nc + 15) / 16) * 16;
    int *mark = reinterpret_cast<int *>(p);
    int64_t *ro = row_out ? row_out + b * k : nullptr;
    int64_t *co = col_out ? col_out + b * k : nullptr;
    auto emit = [&](const auto &c4r) { lsa_emit_wave(c4r, nr0, nc0, mark, ro, co, nullptr); };
    int status;
    if (LDS_COST) {
        status = lsa_stage_wave<IT, CT>(Cb, s1, s2, nr0, nc0, maximize != 0, cost);
        if (status == ASG_OK) status = solve_emit_cpl<CPL>(DenseCost<CT>{cost, nc}, nr, nc, emit);
    } else {
        status = lsa_check_wave<IT>(Cb, s1, s2, nr0, nc0, maximize != 0);
        if (status == ASG_OK)
            status = solve_emit_cpl<CPL>(GlobalCost<IT>{Cb, s1, s2, tr, maximize != 0}, nr, nc, emit);
    }
    const int lane = threadIdx.x;
    if (status != ASG_OK) {
        for (int r = lane; r < k; r += kWave) {
            if (ro) ro[r] = -1;
            if (co) co[r] = -1;
        }
    }
    if (lane == 0 && status_out) status_out[b] = status;
}

static size_t lsa_scratch_bytes(int nr0) { return sizeof(int) * nr0 + 64; }

// float32 problems up to 64 x 64 (working orientation): the working matrix lives in the
// wave's registers (RegCostF32), so residency is set by registers alone (no LDS)
#ifndef ASG_LSA_REG_WAVES
#define ASG_LSA_REG_WAVES 5
#endif
// Problems (waves) per workgroup of the register-resident kernels.  One-wave workgroups cap
// a CU at its 16 resident workgroups = 4 waves per SIMD whatever the register budget allows;
// four waves per workgroup let the 88-VGPR solver run at its 5 waves per SIMD.
#ifndef ASG_LSA_WPB
#define ASG_LSA_WPB 4
#endif
constexpr int kLsaWpb = ASG_LSA_WPB;
static dim3 lsa_reg_grid(int64_t B) { return dim3((unsigned)((B + kLsaWpb - 1) / kLsaWpb)); }
// this wave's problem index (wave-uniform); >= B for the idle waves of the last workgroup
__device__ __forceinline__ int64_t lsa_reg_problem() {
    return (int64_t)blockIdx.x * kLsaWpb + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}
__global__ void __launch_bounds__(64 * kLsaWpb) __attribute__((amdgpu_waves_per_eu(ASG_LSA_REG_WAVES))) lsa_reg_kernel(const float *C, int64_t s0, int64_t s1, int64_t s2, int nr0,
                                                     int nc0, int maximize, int64_t *row_out, int64_t *col_out,
                                                     int32_t *status_out, int64_t B) {
    __shared__ int s_mark[kLsaWpb][64];
    const int64_t b = lsa_reg_problem();
    if (b >= B) return;
    int *mark = s_mark[threadIdx.x >> 6];
    const bool tr = nc0 < nr0;
    const int nr = tr ? nc0 : nr0, nc = tr ? nr0 : nc0;
    const int k = nr;
    int64_t *ro = row_out ? row_out + b * k : nullptr;
    int64_t *co = col_out ? col_out + b * k : nullptr;
    RegCostF32 rc;
    int status = lsa_stage_regs<float>(C + b * s0, s1, s2, nr0, nc0, maximize != 0, rc);
    if (status == ASG_OK) {
        int c4r[1];
        status = lsa_solve_reg64(rc, nr, nc, c4r);
        if (status == ASG_OK) lsa_emit_wave(c4r, nr0, nc0, mark, ro, co, nullptr);
    }
    const int lane = threadIdx.x & (kWave - 1);
    if (status != ASG_OK) {
        for (int r = lane; r < k; r += kWave) {
            if (ro) ro[r] = -1;
            if (co) co[r] = -1;
        }
    }
    if (lane == 0 && status_out) status_out[b] = status;
}

template <typename IT, typename CT>
static hipError_t launch_lsa_t(const IT *C, const int64_t st[3], int64_t B, int nr0, int nc0, int maximize,
                               int64_t *row_out, int64_t *col_out, int32_t *status_out, hipStream_t s) {
    const int nr = nc0 < nr0 ? nc0 : nr0, nc = nc0 < nr0 ? nr0 : nc0;
    const size_t cost_bytes = ((sizeof(CT) * (size_t)nr * nc + 15) / 16) * 16;
    const size_t scratch = lsa_scratch_bytes(nr0);
    if (std::is_same<IT, float>::value && nc <= 64) {
        hipLaunchKernelGGL(lsa_reg_kernel, lsa_reg_grid(B), dim3(64 * kLsaWpb), 0, s, reinterpret_cast<const float *>(C),
                           st[0], st[1], st[2], nr0, nc0, maximize, row_out, col_out, status_out, B);
    } else if (cost_bytes <= kLdsCostBudget) {
#define L_(CPL)                                                                                                   \
    hipLaunchKernelGGL((lsa_batched_kernel<CPL, IT, CT, true>), dim3(B), dim3(64), cost_bytes + scratch, s, C, \
                       st[0], st[1], st[2], nr0, nc0, maximize, row_out, col_out, status_out)
        ASG_DISPATCH_CPL(nc, L_)
#undef L_
    } else {
#define L_(CPL)                                                                                                 \
    hipLaunchKernelGGL((lsa_batched_kernel<CPL, IT, CT, false>), dim3(B), dim3(64), scratch, s, C, st[0], st[1], \
                       st[2], nr0, nc0, maximize, row_out, col_out, status_out)
        ASG_DISPATCH_CPL(nc, L_)
#undef L_
    }
    return hipGetLastError();
}

hipError_t launch_lsa_batched(const void *C, int dtype, const int64_t strides[3], int64_t B, int nr, int nc,
                              int maximize, int64_t *row_out, int64_t *col_out, int32_t *status_out,
                              hipStream_t s) {
    if (dtype == ASG_F32)
        return launch_lsa_t<float, float>(static_cast<const float *>(C), strides, B, nr, nc, maximize, row_out,
                                          col_out, status_out, s);
    return launch_lsa_t<double, double>(static_cast<const double *>(C), strides, B, nr, nc, maximize, row_out,
                                        col_out, status_out, s);
}

// ------------------------------------------------------------------------------------
// SequentialAssignmentProblemSelector (sap_selectors.py:52-98), n <= m <= 64, fused:
// noise of std mean|Q| * eps * 2 added in registers while the column is staged, then the
// register-resident LSA (maximize).  The reference runs, per env on the host: abs, mean,
// ones * avg * eps * 2, torch.normal, +=, scipy.
// ------------------------------------------------------------------------------------
// kWarm: `duals` [B][64] float64 holds each env's column duals from its previous selection --
// the fast path's warm start (lsa_fast_reg64) -- and receives this selection's (NaN when the
// fast path did not finish: the next call starts that env cold)
template <bool kCount, bool kDense64, bool kWarm = false>
__global__ void __launch_bounds__(64 * kLsaWpb) __attribute__((amdgpu_waves_per_eu(ASG_LSA_REG_WAVES))) sap_select_kernel(const float *q, int64_t q0, int64_t q1, int64_t q2, int n,
                                                        int m, float epsilon, uint64_t seed, uint32_t counter,
                                                        int64_t env_base, float *col_out, int64_t *act_out,
                                                        int32_t *status_out, int32_t *steps_out, int64_t B,
                                                        double *duals = nullptr, int warm = 0) {
    __shared__ uint64_t s_slot[kLsaWpb][64];
    const int64_t b = lsa_reg_problem();
    if (b >= B) return;
    sap_select_one<kCount, kDense64, kWarm>(q, q0, q1, q2, n, m, epsilon, seed, counter, env_base, b, col_out, act_out,
                                            status_out, steps_out, duals, warm, s_slot[threadIdx.x >> 6]);
}

// the noisy Q the selector solves (Q + its noise, as sap_stage forms it): parity tooling,
// the SAP selection at epsilon > 0 is checked against scipy on exactly this matrix
__global__ void __launch_bounds__(64 * kLsaWpb) sap_noise_kernel(const float *q, int64_t q0, int64_t q1, int64_t q2,
                                                                 int n, int m, float epsilon, uint64_t seed,
                                                                 uint32_t counter, int64_t env_base, float *q_out,
                                                                 int32_t *status_out, int64_t B) {
    const int64_t b = lsa_reg_problem();
    if (b >= B) return;
    RegCostF32 rc;
    const int status = sap_stage<false>(q, q0, q1, q2, n, m, epsilon, seed, counter, env_base, b, rc);
    const int lane = threadIdx.x & (kWave - 1);
    float *o = q_out + b * n * m + lane;
    if (lane < m) {
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            if (i < n) o[i * m] = -rc.lo[i];
            if (i + 32 < n) o[(i + 32) * m] = -rc.hi[i];
        }
    }
    if (lane == 0 && status_out) status_out[b] = status;
}

hipError_t launch_sap_noise(const float *q, const int64_t qs[3], int64_t B, int n, int m, float epsilon, uint64_t seed,
                            uint32_t counter, int64_t env_base, float *q_out, int32_t *status_out, hipStream_t s) {
    hipLaunchKernelGGL(sap_noise_kernel, lsa_reg_grid(B), dim3(64 * kLsaWpb), 0, s, q, qs[0], qs[1], qs[2], n, m,
                       epsilon, seed, counter, env_base, q_out, status_out, B);
    return hipGetLastError();
}

// occupancy experiments (compile-time, like ASG_SAP_STAGE_ONLY): -DASG_SAP_LDS_PAD=<bytes> of
// unused dynamic LDS per 4-wave workgroup caps the resident waves (e.g. 81920: 2 workgroups = 2
// waves per SIMD) -- the rollout kernel's residency, to price an LSA fused into it; 0 = none
#ifndef ASG_SAP_LDS_PAD
#define ASG_SAP_LDS_PAD 0
#endif
static_assert(ASG_SAP_LDS_PAD >= 0 && ASG_SAP_LDS_PAD <= 160 * 1024, "ASG_SAP_LDS_PAD exceeds the CU's LDS");
static constexpr size_t sap_lds_pad() { return (size_t)ASG_SAP_LDS_PAD; }

hipError_t launch_sap_select(const float *q, const int64_t qs[3], int64_t B, int n, int m, float epsilon,
                             uint64_t seed, uint32_t counter, int64_t env_base, float *col_out, int32_t *status_out,
                             int32_t *steps_out, hipStream_t s, int64_t *act_out, double *duals, int warm) {
    const dim3 grid = lsa_reg_grid(B);
    const size_t pad = sap_lds_pad();
    // the rollout's Q rows ([B][64][64] contiguous): the unguarded staging instance
    const bool d64 = n == 64 && m == 64 && qs[2] == 1 && qs[1] == 64 && (reinterpret_cast<uintptr_t>(q) & 3) == 0;
#define SAP_L(C, D)                                                                                                 \
    hipLaunchKernelGGL((sap_select_kernel<C, D>), grid, dim3(64 * kLsaWpb), pad, s, q, qs[0], qs[1], qs[2], n, m, \
                       epsilon, seed, counter, env_base, col_out, act_out, status_out, steps_out, B, nullptr, 0)
#define SAP_LW(C, D)                                                                                                   \
    hipLaunchKernelGGL((sap_select_kernel<C, D, true>), grid, dim3(64 * kLsaWpb), pad, s, q, qs[0], qs[1], qs[2], n, m, \
                       epsilon, seed, counter, env_base, col_out, act_out, status_out, steps_out, B, duals, warm)
    if (duals) {  // warm-started fast path (square problems; the runner's selection)
        if (steps_out) {
            if (d64) SAP_LW(true, true);
            else SAP_LW(true, false);
        } else {
            if (d64) SAP_LW(false, true);
            else SAP_LW(false, false);
        }
#undef SAP_LW
    } else if (steps_out) {
        if (d64) SAP_L(true, true);
        else SAP_L(true, false);
    } else {
        if (d64) SAP_L(false, true);
        else SAP_L(false, false);
    }
#undef SAP_L
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// bids_as_actions with the ContinuousActionSelector (ippo_sap.yaml), n <= m <= 64, fused: env
// b's agent outputs (the rollout kernel's Q rows) -> softmax over the tasks (BasicMAC.forward
// with agent_output_type "pi_logits", basic_controller.py:37-46) -> softmax over the agents
// (softmax_agent_inputs, bet_selectors.py:13) -> th.normal(x, std) = x + std z (bet_selectors.py:
// 15-20; z from Philox keyed by (seed, global env, call)) -> the bids, stored as the batch's
// actions row -> LSA(bids, maximize) = the env's assignments for its next step
// (mock_constellation_env.py:121-122), kept in the handle for asg_step / asg_step_forward.
// ------------------------------------------------------------------------------------
// ASG_BIDS_WAVES: waves per SIMD the kernel is compiled for (0: the register allocator's choice,
// 110 VGPRs at 4 waves; 5: 96 VGPRs with 26 spilled, 0.489 vs 0.498 ms, r5 A/B)
#ifndef ASG_BIDS_WAVES
#define ASG_BIDS_WAVES 5
#endif
// The row softmax's per-row max and sum over the 64 lanes, 16 rows at a time: rows 8g + j (a[j])
// and 8g + j + 32 (b[j]), j < 8, folded by a transposing butterfly -- v_permlane32_swap /
// v_permlane16_swap hand each lane its partner's copy of the rows it keeps (one instruction per
// pair), then row_mirror / row_half_mirror DPP, then a quad reduction -- 17 cross-lane steps for
// 16 rows instead of 16 wave reductions of 6 DPP steps and a broadcast each (one row-softmax pass
// priced at 0.076 ms of the kernel's 0.497, profiles/r6_bids_rowsm_s25.txt).  Lane l ends with
// row 8g + (l >> 2 & 7) + 32 (l >> 5) reduced over all lanes: row_lane16(r) is where row r is.
#ifndef ASG_BIDS_ROW_GROUPS
#define ASG_BIDS_ROW_GROUPS 1
#endif
__device__ __forceinline__ float f_of(uint32_t u) { return __builtin_bit_cast(float, u); }
__device__ __forceinline__ uint32_t u_of(float f) { return __builtin_bit_cast(uint32_t, f); }
template <class Op>
__device__ __forceinline__ float rows16_reduce(const float (&a)[8], const float (&b)[8], Op op) {
    const int lane = threadIdx.x & 63;
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // lanes < 32 keep row 8g + j, lanes >= 32 row 8g + j + 32
        const auto r = __builtin_amdgcn_permlane32_swap(u_of(a[j]), u_of(b[j]), false, false);
        t[j] = op(f_of(r[0]), f_of(r[1]));
    }
    float u[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // + 4 (lane bit 4)
        const auto r = __builtin_amdgcn_permlane16_swap(u_of(t[j]), u_of(t[j + 4]), false, false);
        u[j] = op(f_of(r[0]), f_of(r[1]));
    }
    const bool b3 = (lane & 8) != 0, b2 = (lane & 4) != 0;
    float w[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // + 2 (lane bit 3): partner 15 - i in the 16-lane row
        const float keep = b3 ? u[j + 2] : u[j], send = b3 ? u[j] : u[j + 2];
        w[j] = op(keep, f_of((uint32_t)__builtin_amdgcn_update_dpp(0, (int)u_of(send), 0x140, 0xf, 0xf, false)));
    }
    // + 1 (lane bit 2): partner 7 - i in the 8-lane half row
    const float keep = b2 ? w[1] : w[0], send = b2 ? w[0] : w[1];
    float v = op(keep, f_of((uint32_t)__builtin_amdgcn_update_dpp(0, (int)u_of(send), 0x141, 0xf, 0xf, false)));
    // the quad holds four disjoint 16-lane partials of the same row
    v = op(v, f_of((uint32_t)__builtin_amdgcn_update_dpp(0, (int)u_of(v), 0x4e, 0xf, 0xf, false)));
    v = op(v, f_of((uint32_t)__builtin_amdgcn_update_dpp(0, (int)u_of(v), 0xb1, 0xf, 0xf, false)));
    return v;
}
// the lane holding row r (r mod 32 in [8g, 8g + 8)) after rows16_reduce of its group
__device__ __forceinline__ constexpr int row_lane16(int r) { return 32 * (r >> 5) + 4 * (r & 7); }

// kCount: the instrumented instance (bench.py's efficiency figure): steps_out[b] = the env's
// augmenting-path steps, fast path in bits 0..15, scipy-exact solver above (as asg_sap_select)
template <bool kCount>
__global__ void __launch_bounds__(64 * kLsaWpb)
#if ASG_BIDS_WAVES
__attribute__((amdgpu_waves_per_eu(ASG_BIDS_WAVES)))
#endif
bids_select_kernel(const float *q, int64_t q0, int64_t q1, int64_t q2, int n, int m, int row_sm, int col_sm,
                   float stdv, uint64_t seed, uint32_t counter, int64_t env_base, float *bids, int64_t o0,
                   int64_t o1, int64_t o2, int *assign, int *env_err, int64_t B, int32_t *steps_out = nullptr) {
    __shared__ uint64_t s_slot[kLsaWpb][64];
    const int64_t b = lsa_reg_problem();
    if (b >= B) return;
    const int lane = threadIdx.x & (kWave - 1);
    const bool lv = lane < m;
    asm volatile("" : "+s"(q0), "+s"(q1), "+s"(q2), "+s"(o0), "+s"(o1), "+s"(o2));
    RegColPin<32> rc;  // column `lane` of the env's matrix, rows 0..31 in lo, 32..63 in hi
    {
        const float *col = q + b * q0 + (int64_t)lane * q2;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            rc.lo[i] = (lv && i < n) ? col[i * q1] : 0.0f;
            rc.hi[i] = (lv && i + 32 < n) ? col[(i + 32) * q1] : 0.0f;
        }
    }
    // f(x, i) applied to every row i < n of the column (rows at compile-time register slots)
    auto each_row = [&](auto f) {
#pragma unroll
        for (int i = 0; i < 32; ++i)
            if (i < n) rc.lo[i] = f(rc.lo[i], i);
#pragma unroll
        for (int i = 0; i < 32; ++i)
            if (i + 32 < n) rc.hi[i] = f(rc.hi[i], i + 32);
    };
    // exp as v_exp_f32 of x log2(e) (x = y - max <= 0: relative error <= |x| 2^-24 + 1 ulp; torch's
    // expf is within 1 ulp): the accurate expf unrolled over the 64 rows spilled at any budget
#ifdef ASG_BIDS_TIMING_RS2  // timing only: one extra row-softmax pass, its results discarded
    if (row_sm) {
        each_row([&](float x, int) {
            const float mx = wave_allreduce(lv ? x : -__builtin_inff(), [](float a, float c) { return fmaxf(a, c); });
            const float ex = lv ? __expf(x - mx) : 0.0f;
            const float sum = wave_allreduce(ex, [](float a, float c) { return a + c; });
            const float r = ex / sum;
            asm volatile("" ::"v"(r));
            return x;
        });
    }
#endif
    if (row_sm && ASG_BIDS_ROW_GROUPS) {  // softmax(dim = -1) of each agent's row: exp(x - max) / sum
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            float a[8], bb[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                a[j] = lv ? rc.lo[8 * g + j] : -__builtin_inff();
                bb[j] = lv ? rc.hi[8 * g + j] : -__builtin_inff();
            }
            const float mx = rows16_reduce(a, bb, [](float x, float y) { return fmaxf(x, y); });
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float ma = f_of((uint32_t)__builtin_amdgcn_readlane((int)u_of(mx), row_lane16(8 * g + j)));
                const float mb = f_of((uint32_t)__builtin_amdgcn_readlane((int)u_of(mx), row_lane16(8 * g + j + 32)));
                a[j] = lv ? __expf(rc.lo[8 * g + j] - ma) : 0.0f;
                bb[j] = lv ? __expf(rc.hi[8 * g + j] - mb) : 0.0f;
            }
            const float sm = rows16_reduce(a, bb, [](float x, float y) { return x + y; });
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float sa = f_of((uint32_t)__builtin_amdgcn_readlane((int)u_of(sm), row_lane16(8 * g + j)));
                const float sb = f_of((uint32_t)__builtin_amdgcn_readlane((int)u_of(sm), row_lane16(8 * g + j + 32)));
                if (8 * g + j < n) rc.lo[8 * g + j] = a[j] / sa;
                if (8 * g + j + 32 < n) rc.hi[8 * g + j] = bb[j] / sb;
            }
        }
    } else if (row_sm) {  // softmax(dim = -1) of each agent's row: exp(x - max) / sum, as torch
        each_row([&](float x, int) {
            const float mx = wave_allreduce(lv ? x : -__builtin_inff(), [](float a, float c) { return fmaxf(a, c); });
            const float ex = lv ? __expf(x - mx) : 0.0f;
            const float sum = wave_allreduce(ex, [](float a, float c) { return a + c; });
            return ex / sum;
        });
    }
    if (col_sm) {  // softmax(dim = 1): over the agents, lane-local
        float mx = -__builtin_inff(), sum = 0.0f;
        each_row([&](float x, int) {
            mx = fmaxf(mx, x);
            return x;
        });
        each_row([&](float x, int) {
            const float ex = __expf(x - mx);
            sum += ex;
            return ex;
        });
        each_row([&](float x, int) { return x / sum; });
    }
    if (stdv > 0.0f) {  // th.normal(mean, std): mean + std * z (std = 0 keeps the means exactly)
        const EnvKey key = env_key(seed, env_base + b);
        constexpr float k2m24 = 5.9604644775390625e-08f;  // 2^-24
        constexpr float k2pi = 6.283185307179586f;
#pragma unroll
        for (int i4 = 0; i4 < 16; ++i4) {  // rows 4 i4 .. 4 i4 + 3 of this column (rows >= n unused)
            const u32x4 r = philox4x32_10(u32x4{(uint32_t)lane, (uint32_t)i4, kCtrBidsNoise, counter}, key.k0, key.k1);
            const float u1a = (float)((r.x >> 8) + 1u) * k2m24, u2a = (float)(r.y >> 8) * k2m24;
            const float u1b = (float)((r.z >> 8) + 1u) * k2m24, u2b = (float)(r.w >> 8) * k2m24;
            const float ra = __builtin_sqrtf(-2.0f * __logf(u1a)), rb = __builtin_sqrtf(-2.0f * __logf(u1b));
            const float z[4] = {ra * __cosf(k2pi * u2a), ra * __sinf(k2pi * u2a), rb * __cosf(k2pi * u2b),
                                rb * __sinf(k2pi * u2b)};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int i = 4 * i4 + k;
                if (i < 32) rc.lo[i] = rc.lo[i] + stdv * z[k];
                else rc.hi[i - 32] = rc.hi[i - 32] + stdv * z[k];
            }
        }
    }
    // the bids: the actions the batch stores (one 64-float row per store instruction); scipy
    // maximize on the float64 bids: NaN or +inf (-inf once negated) is invalid
    int bad = 0;
    {
        float *o = bids + b * o0 + (int64_t)lane * o2;
        each_row([&](float x, int i) {
            if (lv) o[i * o1] = x;
            bad |= lv & ((x != x) | (x == __builtin_inff()));
            return x;
        });
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        rc.lo[i] = (lv && i < n) ? -rc.lo[i] : 0.0f;
        rc.hi[i] = (lv && i + 32 < n) ? -rc.hi[i] : 0.0f;
    }
    int status = __builtin_amdgcn_readfirstlane(wave_or_i32(bad)) ? ASG_E_LSA_INVALID : ASG_OK;
    int c4r[1] = {-1};
    int nfast = 0, nsteps = 0;
    bool done = false;
    if (ASG_SAP_FAST && status == ASG_OK && n == m)
        done = lsa_fast_reg64<decltype(rc), kCount>(rc, n, c4r, &nfast, s_slot[threadIdx.x >> 6]) == ASG_OK;
    if (status == ASG_OK && !done) status = lsa_solve_reg64<decltype(rc), kCount>(rc, n, m, c4r, &nsteps);
    if (lane < n) assign[b * n + lane] = status == ASG_OK ? c4r[0] : -1;
    if (status != ASG_OK && lane == 0) atomicCAS(env_err, 0, status);
    if (kCount && lane == 0 && steps_out) steps_out[b] = nfast | (nsteps << 16);
}

hipError_t launch_bids_select(const float *q, const int64_t qs[3], int64_t B, int n, int m, int row_sm, int col_sm,
                              float stdv, uint64_t seed, uint32_t counter, int64_t env_base, float *bids,
                              const int64_t os[3], int *assign, int *env_err, hipStream_t s, int32_t *steps_out) {
    if (steps_out)
        hipLaunchKernelGGL(bids_select_kernel<true>, lsa_reg_grid(B), dim3(64 * kLsaWpb), 0, s, q, qs[0], qs[1], qs[2],
                           n, m, row_sm, col_sm, stdv, seed, counter, env_base, bids, os[0], os[1], os[2], assign,
                           env_err, B, steps_out);
    else
        hipLaunchKernelGGL(bids_select_kernel<false>, lsa_reg_grid(B), dim3(64 * kLsaWpb), 0, s, q, qs[0], qs[1],
                           qs[2], n, m, row_sm, col_sm, stdv, seed, counter, env_base, bids, os[0], os[1], os[2],
                           assign, env_err, B, nullptr);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// beta_hat = beta - lambda * T_trans[prev_i, j] * (beta > 1e-12)   (mock :250-270)
// ------------------------------------------------------------------------------------
template <typename BT>
__global__ void beta_hat_kernel(const BT *beta, int64_t b0, int64_t b1, int64_t b2, const int64_t *prev, int64_t p0,
                                int64_t p1, int64_t B, int n, int m, const double *T_trans, double lambda_,
                                double *out) {
    const int64_t total = B * n * m;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int j = (int)(idx % m);
        const int64_t bi = idx / m;
        const int i = (int)(bi % n);
        const int64_t b = bi / n;
        const double x = (double)beta[b * b0 + i * b1 + j * b2];
        const int64_t p = prev[b * p0 + i * p1];
        const double tt = T_trans ? T_trans[p * m + j] : (j == p ? 0.0 : 1.0);
        out[idx] = x - lambda_ * (tt * (x > 1e-12 ? 1.0 : 0.0));
    }
}

hipError_t launch_beta_hat(const void *beta, int dtype, const int64_t bs[3], const int64_t *prev,
                           const int64_t ps[2], int64_t B, int n, int m, const double *T_trans, double lambda_,
                           double *out, hipStream_t s) {
    const int64_t total = B * n * m;
    const int64_t blocks = total == 0 ? 1 : (total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192;
    if (dtype == ASG_F32)
        hipLaunchKernelGGL(beta_hat_kernel<float>, dim3(blocks), dim3(256), 0, s, static_cast<const float *>(beta),
                           bs[0], bs[1], bs[2], prev, ps[0], ps[1], B, n, m, T_trans, lambda_, out);
    else
        hipLaunchKernelGGL(beta_hat_kernel<double>, dim3(blocks), dim3(256), 0, s,
                           static_cast<const double *>(beta), bs[0], bs[1], bs[2], prev, ps[0], ps[1], B, n, m,
                           T_trans, lambda_, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// HAASelector (non_rl_selectors.py:19-50): col = LSA(beta_hat(beta, prev), maximize)[1]
// The working matrix -beta_hat is formed on the fly from the f32 beta staged in LDS, so
// a 64x64 problem needs 16 KiB of LDS instead of 32.
// ------------------------------------------------------------------------------------
struct HaaCost {
    static constexpr bool kInMemory = true;
    const float *beta;  // [n][m] in LDS (rs = m, cs = 1) or in place in global memory
    int64_t rs, cs;
    const int *prev;    // LDS [n]
    const double *T_trans;
    double lambda_;
    int m;
    __device__ double operator()(int i, int j) const {
        const double x = (double)beta[i * rs + j * cs];
        const int p = prev[i];
        const double tt = T_trans ? T_trans[(int64_t)p * m + j] : (j == p ? 0.0 : 1.0);
        return -(x - lambda_ * (tt * (x > 1e-12 ? 1.0 : 0.0)));
    }
};

template <int CPL, bool STAGE>
__global__ void __launch_bounds__(64) haa_select_kernel(const float *beta, int64_t b0, int64_t b1, int64_t b2,
                                                        const int64_t *prev, int64_t p0, int64_t p1, int n, int m,
                                                        const double *T_trans, double lambda_, float *col_out,
                                                        int32_t *status_out) {
    extern __shared__ double s_lsa[];
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    char *p = reinterpret_cast<char *>(s_lsa);
    float *sb = reinterpret_cast<float *>(p);
    if (STAGE) p += ((sizeof(float) * (size_t)n * m + 15) / 16) * 16;
    int *sp = reinterpret_cast<int *>(p);
    int bad = 0;
    for (int idx = lane; idx < n * m; idx += kWave) {
        const int i = idx / m, j = idx - i * m;
        const float x = beta[b * b0 + i * b1 + j * b2];
        if (STAGE) sb[idx] = x;
        bad |= (x != x) || (x == __builtin_inff());  // -(+inf) = -inf is invalid
    }
    for (int i = lane; i < n; i += kWave) sp[i] = (int)prev[b * p0 + i * p1];
    wave_sync();
    float *co = col_out + b * n;
    auto emit = [&](const auto &c4r) { lsa_emit_wave(c4r, n, m, nullptr, nullptr, nullptr, co); };
    int status = wave_or_i32(bad) ? ASG_E_LSA_INVALID : ASG_OK;
    if (status == ASG_OK) {
        const HaaCost acc = STAGE ? HaaCost{sb, m, 1, sp, T_trans, lambda_, m}
                                  : HaaCost{beta + b * b0, b1, b2, sp, T_trans, lambda_, m};
        status = solve_emit_cpl<CPL>(acc, n, m, emit);
    }
    if (status != ASG_OK)
        for (int i = lane; i < n; i += kWave) co[i] = -1.0f;
    if (lane == 0 && status_out) status_out[b] = status;
}

// m <= 64: the beta column of the lane's task and prev_assigns of the lane's agent stay
// in registers; -beta_hat(i, j) is formed per relaxed entry
struct HaaRegCost {
    static constexpr bool kInMemory = false;  // T_trans reads are guarded below
    RegCostF32 beta;  // beta[i][lane], not sign-flipped
    int prev;         // prev_assigns[lane]
    const double *T_trans;
    double lambda_;
    int m;
    __device__ double operator()(int i, int j) const {
        const double x = (double)beta.get(i);
        const int p = __builtin_amdgcn_readlane(prev, i);
        const double tt = T_trans ? (j < m ? T_trans[(int64_t)p * m + j] : 0.0) : (j == p ? 0.0 : 1.0);
        return -(x - lambda_ * (tt * (x > 1e-12 ? 1.0 : 0.0)));
    }
    __device__ double col(int i) const { return (*this)(i, (int)(threadIdx.x & 63)); }
};

__global__ void __launch_bounds__(64 * kLsaWpb) __attribute__((amdgpu_waves_per_eu(ASG_LSA_REG_WAVES))) haa_reg_kernel(const float *beta, int64_t b0, int64_t b1, int64_t b2,
                                                     const int64_t *prev, int64_t p0, int64_t p1, int n, int m,
                                                     const double *T_trans, double lambda_, float *col_out,
                                                     int32_t *status_out, int64_t B) {
    const int64_t b = lsa_reg_problem();
    if (b >= B) return;
    const int lane = threadIdx.x & (kWave - 1);
    HaaRegCost acc;
    // beta_hat is not negated here (the accessor does it): stage with maximize = false,
    // which also rejects NaN; +inf beta (-inf cost) is rejected below
    int status = lsa_stage_regs<float>(beta + b * b0, b1, b2, n, m, false, acc.beta);
    int bad = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i)
        bad |= (acc.beta.lo[i] == __builtin_inff()) | (acc.beta.hi[i] == __builtin_inff());
    if (wave_or_i32(bad)) status = ASG_E_LSA_INVALID;
    acc.prev = lane < n ? (int)prev[b * p0 + lane * p1] : 0;
    acc.T_trans = T_trans;
    acc.lambda_ = lambda_;
    acc.m = m;
    float *co = col_out + b * n;
    if (status == ASG_OK) {
        int c4r[1];
        status = lsa_solve_reg64(acc, n, m, c4r);
        if (status == ASG_OK) lsa_emit_wave(c4r, n, m, nullptr, nullptr, nullptr, co);
    }
    if (status != ASG_OK)
        for (int i = lane; i < n; i += kWave) co[i] = -1.0f;
    if (lane == 0 && status_out) status_out[b] = status;
}

hipError_t launch_haa_select(const float *beta, const int64_t bs[3], const int64_t *prev, const int64_t ps[2],
                             int64_t B, int n, int m, const double *T_trans, double lambda_, float *col_out,
                             int32_t *status_out, hipStream_t s) {
    const size_t cost = ((sizeof(float) * (size_t)n * m + 15) / 16) * 16;
    const size_t rest = ((sizeof(int) * n + 15) / 16) * 16 + 64;
    if (m <= 64) {
        hipLaunchKernelGGL(haa_reg_kernel, lsa_reg_grid(B), dim3(64 * kLsaWpb), 0, s, beta, bs[0], bs[1], bs[2], prev,
                           ps[0], ps[1], n, m, T_trans, lambda_, col_out, status_out, B);
    } else if (cost <= kLdsCostBudget) {
#define L_(CPL)                                                                                                 \
    hipLaunchKernelGGL((haa_select_kernel<CPL, true>), dim3(B), dim3(64), cost + rest, s, beta, bs[0], bs[1], bs[2], \
                       prev, ps[0], ps[1], n, m, T_trans, lambda_, col_out, status_out)
        ASG_DISPATCH_CPL(m, L_)
#undef L_
    } else {
#define L_(CPL)                                                                                                  \
    hipLaunchKernelGGL((haa_select_kernel<CPL, false>), dim3(B), dim3(64), rest, s, beta, bs[0], bs[1], bs[2], prev, \
                       ps[0], ps[1], n, m, T_trans, lambda_, col_out, status_out)
        ASG_DISPATCH_CPL(m, L_)
#undef L_
    }
    return hipGetLastError();
}

}  // namespace asg
