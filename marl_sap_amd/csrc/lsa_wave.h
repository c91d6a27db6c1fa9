// lsa_wave.h -- one wave64 solves one rectangular linear sum assignment problem with
// exactly scipy's shortest-augmenting-path algorithm, tie rule and float64 operation
// order (scipy 1.15.3 `linear_sum_assignment`; restated in SURVEY.md Appendix B), so
// the assignments are bit-identical to the reference's scipy calls
// (mock_constellation_env.py:122, sap_selectors.py:32,90, non_rl_selectors.py:47).
//
// Parallelisation: lane l owns columns j = l + 64*c (c < CPL).  The serial scipy scan
// over `remaining` becomes: every lane relaxes its own columns, then one packed wave
// reduction picks the column the sequential scan would have picked:
//   lowest = min spc over remaining; candidates = remaining columns with spc == lowest;
//   if some candidate is unassigned: the candidate of LARGEST position in `remaining`
//   among the unassigned ones, else the candidate of SMALLEST position.
// `remaining` positions are tracked per column (pos), including scipy's
// swap-with-last removal, so ties resolve exactly as in the sequential code.
//
// The working matrix (already transposed so nr <= nc, and sign-flipped for maximize, as
// scipy does before solving) lives in registers for float32 problems up to 64 x 64
// (RegCostF32), else in LDS, else (large problems) is read in place from global memory.
#pragma once
#include "asg_device.h"

namespace asg {

// Row-major cost matrix in LDS (already transposed / sign-flipped)
template <typename CT>
struct DenseCost {
    static constexpr bool kInMemory = true;
    const CT *c;
    int nc;
    __device__ double operator()(int i, int j) const { return (double)c[(size_t)i * nc + j]; }
};

// Register-resident working matrix of at most 64 x 64 float32 entries: lane l holds
// working column l (rows 0..31 in `lo`, 32..63 in `hi`).  A row index is wave-uniform,
// so the read is two s_set_gpr_idx moves and a select -- no LDS, no memory latency, and
// no LDS budget capping the problems resident per CU.
typedef float f32x32 __attribute__((ext_vector_type(32)));
struct RegCostF32 {
    static constexpr bool kInMemory = false;
    f32x32 lo, hi;
    __device__ __forceinline__ float get(int i) const {
        const int ii = __builtin_amdgcn_readfirstlane(i);
        const float x0 = lo[ii & 31], x1 = hi[ii & 31];
        return ii < 32 ? x0 : x1;
    }
    __device__ __forceinline__ double operator()(int i, int) const { return (double)get(i); }
    __device__ __forceinline__ double col(int i) const { return (double)get(i); }
};

// The same column pinned to physical registers v[BASE .. BASE + 63] (rows 0..31 in lo =
// v[BASE .. BASE + 31], 32..63 in hi right after it), so a row read is ONE indexed move
// (s_set_gpr_idx_on row; v_mov_b32 from v[BASE]) with no select, and the IR never indexes
// the vector dynamically (a variable index into a column that lives across loops keeps it in
// scratch): the column is an asm operand, whole.  For the multi-problem kernels, whose
// columns are loop-carried.
#define ASG_PIN_READ(B, LO, HI)                                                                  \
    asm("s_set_gpr_idx_on %1, gpr_idx(SRC0)\n\tv_mov_b32 %0, v" #B "\n\ts_set_gpr_idx_off"     \
        : "=v"(x)                                                                               \
        : "s"(ii), "{v[" #LO "]}"(lo), "{v[" #HI "]}"(hi))
template <int BASE>
struct RegColPin {
    static constexpr bool kInMemory = false;
    f32x32 lo, hi;
    __device__ __forceinline__ float get(int i) const {
        const int ii = __builtin_amdgcn_readfirstlane(i);
        float x;
        if constexpr (BASE == 32) ASG_PIN_READ(32, 32:63, 64:95);
        else if constexpr (BASE == 16) ASG_PIN_READ(16, 16:47, 48:79);
        else if constexpr (BASE == 24) ASG_PIN_READ(24, 24:55, 56:87);
        else if constexpr (BASE == 40) ASG_PIN_READ(40, 40:71, 72:103);
        else if constexpr (BASE == 104) ASG_PIN_READ(104, 104:135, 136:167);
        else if constexpr (BASE == 64) ASG_PIN_READ(64, 64:95, 96:127);
        else if constexpr (BASE == 128) ASG_PIN_READ(128, 128:159, 160:191);
        else {
            static_assert(BASE == 192, "a pinned base with an instance here");
            ASG_PIN_READ(192, 192:223, 224:255);
        }
        return x;
    }
    __device__ __forceinline__ double col(int i) const { return (double)get(i); }
};
#undef ASG_PIN_READ

// Load the lane's working column (scipy orientation: transposed when nr0 > nc0, negated
// for maximize) into registers.  Returns ASG_E_LSA_INVALID (wave uniform) when an entry
// is NaN or -inf after the sign flip.
template <typename IT>
__device__ int lsa_stage_regs(const IT *C, int64_t rs, int64_t cs, int nr0, int nc0, bool maximize,
                              RegCostF32 &rc) {
    const int lane = threadIdx.x & (kWave - 1);
    const bool tr = nc0 < nr0;
    const int nr = tr ? nc0 : nr0, nc = tr ? nr0 : nc0;
    const int64_t istride = tr ? cs : rs, jstride = tr ? rs : cs;
    const IT *col = C + (int64_t)lane * jstride;
    int bad = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        float a = 0.0f, b = 0.0f;
        if (lane < nc && i < nr) a = (float)col[i * istride];
        if (lane < nc && i + 32 < nr) b = (float)col[(i + 32) * istride];
        if (maximize) {
            a = -a;
            b = -b;
        }
        bad |= (a != a) | (b != b) | (a == -__builtin_inff()) | (b == -__builtin_inff());
        rc.lo[i] = a;
        rc.hi[i] = b;
    }
    return wave_or_i32(bad) ? ASG_E_LSA_INVALID : ASG_OK;
}

// Solve on the working matrix acc(i, j), i < nr <= nc <= 64*CPL (scipy's orientation).
// All per-row and per-column state lives in registers, distributed over the lanes
// (column j / row r in lane j%64, slot j/64); only the cost matrix may be in memory.
// Each augmenting-path step is: relax the lane's columns in float64 (scipy's operation
// order), one int32 min-reduction of the float32-rounded keys plus a ballot -- which
// settles the step whenever a single column attains the minimum key -- and otherwise the
// exact float64 minimum and scipy's tie rule by packed-key reduction.  Control flow is
// wave-uniform throughout (row, column and position indices are scalars).
// Returns 0 or ASG_E_LSA_INFEASIBLE; col4row[c] holds the column assigned to row
// lane + 64c.  All 64 lanes must call it with identical arguments.
template <int CPL, class Acc>
__device__ int lsa_solve_wave(const Acc &acc, int nr, int nc, int (&col4row)[CPL]) {
    const int lane = threadIdx.x & (kWave - 1);
    double v[CPL], u[CPL];
    int r4c[CPL], path[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
        v[c] = 0.0;
        u[c] = 0.0;
        r4c[c] = -1;
        path[c] = -1;
        col4row[c] = -1;
    }
    for (int cur = 0; cur < nr; ++cur) {
        double spc[CPL];
        int pos[CPL];  // position in scipy's `remaining`, -1 once scanned (or absent)
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int j = lane + kWave * c;
            spc[c] = __builtin_inf();
            pos[c] = (j < nc) ? (nc - 1 - j) : -1;  // remaining[it] = nc - it - 1
        }
        int nrem = nc;
        double minv = 0.0;
        int i = cur, sink = -1;
        bool infeasible = false;
        do {
            i = __builtin_amdgcn_readfirstlane(i);
            const double ui = lane_get(u, i);
            float key[CPL];
            float kl = __builtin_inff();
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int j = lane + kWave * c;
                // branch-free over the lane's columns: scanned / absent ones are relaxed
                // too but neither updated nor keyed (+inf keys: a remaining column at
                // +inf ties with them and takes the exact path)
                const bool rem = pos[c] >= 0;
                // never read past a matrix in memory; register columns are always valid
                const double cij = (!Acc::kInMemory || j < nc) ? acc(i, j) : 0.0;
                const double r = ((minv + cij) - ui) - v[c];
                const bool upd = rem && r < spc[c];
                spc[c] = upd ? r : spc[c];
                path[c] = upd ? i : path[c];
                key[c] = rem ? (float)spc[c] : __builtin_inff();
                kl = c == 0 ? key[0] : __builtin_fminf(kl, key[c]);
            }
            const float kmin = wave_min_f32_nonan(kl);
            uint64_t cmsk[CPL];
            int total = 0;
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                cmsk[c] = __ballot(key[c] == kmin);
                total += __popcll(cmsk[c]);
            }
            if (total == 0) return ASG_E_LSA_INVALID;  // NaN keys (see lsa_solve_reg64)
            // first candidate (the selection when it is the only one)
            int src0 = 0, c0 = 0;
#pragma unroll
            for (int c = CPL - 1; c >= 0; --c) {
                if (cmsk[c] != 0) {
                    src0 = __builtin_ctzll(cmsk[c]);
                    c0 = c;
                }
            }
            double val0 = 0.0;
            int pos0 = 0;
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                if (c == c0) {
                    const uint64_t sb = __builtin_bit_cast(uint64_t, spc[c]);
                    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)sb, src0);
                    const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(sb >> 32), src0);
                    val0 = __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
                    pos0 = __builtin_amdgcn_readlane(pos[c], src0);
                }
            }
            double lowest = val0;
            int jsel = src0 + kWave * c0, psel = pos0;
            if (total != 1) {
                // Several columns share the minimum key.  Usually they hold exactly equal
                // float64 values (scipy's tie case: zero reduced costs, frequent with
                // correlated Q-values): check that against the first candidate's value,
                // then apply scipy's tie rule with one 32-bit max-reduction.  Otherwise
                // (distinct float64 values that round to one float32) take the exact
                // float64 minimum first.
                bool all_equal = true;
#pragma unroll
                for (int c = 0; c < CPL; ++c) all_equal &= (__ballot(spc[c] != val0) & cmsk[c]) == 0;
                if (!all_equal) {
                    double lo = __builtin_inf();
#pragma unroll
                    for (int c = 0; c < CPL; ++c)
                        if (pos[c] >= 0) lo = spc[c] < lo ? spc[c] : lo;
                    const uint64_t lb = __builtin_bit_cast(uint64_t, wave_min_f64(lo));  // uniform: pin to SGPRs
                    const uint32_t l0 = __builtin_amdgcn_readfirstlane((uint32_t)lb);
                    const uint32_t l1 = __builtin_amdgcn_readfirstlane((uint32_t)(lb >> 32));
                    lowest = __builtin_bit_cast(double, (uint64_t)l0 | ((uint64_t)l1 << 32));
                }
                // scipy's tie rule as a max-reduced 32-bit key over the candidates
                // (remaining columns at `lowest`):
                //   unassigned: 2^31 | pos        (the LARGEST position wins)
                //   assigned:   2^30 - pos        (else the SMALLEST position)
                uint32_t tk = 0;
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    const bool cand = all_equal ? ((cmsk[c] >> lane) & 1) != 0 : (pos[c] >= 0 && spc[c] == lowest);
                    const uint32_t k = (r4c[c] == -1) ? (0x80000000u | (uint32_t)pos[c])
                                                      : ((1u << 30) - (uint32_t)pos[c]);
                    tk = (cand && k > tk) ? k : tk;
                }
                tk = __builtin_amdgcn_readfirstlane(wave_max_u32(tk));
                psel = (tk >> 31) ? (int)(tk & 0x7fffffffu) : (int)((1u << 30) - tk);
                // positions are distinct over the remaining columns: the owner is unique
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    const uint64_t msk = __ballot(pos[c] == psel);
                    if (msk != 0) jsel = __builtin_ctzll(msk) + kWave * c;
                }
            }
            const int last = nrem - 1;
            // remaining[index] = remaining[--num_remaining]
#pragma unroll
            for (int c = 0; c < CPL; ++c)
                pos[c] = (lane + kWave * c == jsel) ? -1 : (pos[c] == last ? psel : pos[c]);
            --nrem;
            minv = lowest;
            const int owner = lane_get(r4c, jsel);
            // scipy: minVal == INFINITY (compared on the bits: a scalar compare)
            infeasible = __builtin_bit_cast(uint64_t, lowest) == 0x7ff0000000000000ull;
            if (owner == -1) sink = jsel;
            i = owner;
        } while (sink == -1 && !infeasible);
        if (infeasible) return ASG_E_LSA_INFEASIBLE;
        // dual update (scipy: u[cur] += minv; u[r] += minv - spc[col4row[r]] for the
        // other visited rows; v[j] -= minv - spc[j] for the scanned columns).  A row
        // r != cur was visited iff its matched column col4row[r] was scanned.
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int r = lane + kWave * c;
            const int jm = col4row[c];
            // gather (scanned, spc) of column jm from its owner lane; a column of the
            // matrix was scanned iff it left `remaining` (pos == -1)
            double spc_j = 0.0;
            int sc_j = 0;
#pragma unroll
            for (int c2 = 0; c2 < CPL; ++c2) {
                const double sv = __shfl(spc[c2], jm & 63, kWave);
                const int sb = __shfl(pos[c2], jm & 63, kWave) < 0;
                if (jm >= 0 && (jm >> 6) == c2) {
                    spc_j = sv;
                    sc_j = sb;
                }
            }
            if (r < nr) {
                if (r == cur) u[c] += minv;
                else if (jm >= 0 && sc_j) u[c] += minv - spc_j;
            }
        }
#pragma unroll
        for (int c = 0; c < CPL; ++c)
            if (pos[c] < 0 && lane + kWave * c < nc) v[c] -= minv - spc[c];
        // augment along path back to cur (uniform loop of lane reads/writes)
        int j = sink;
        while (true) {
            const int pi = lane_get(path, j);
            lane_set(r4c, j, pi);
            const int t = lane_get(col4row, pi);
            lane_set(col4row, pi, j);
            j = t;
            if (pi == cur) break;
        }
    }
    return ASG_OK;
}

// The same algorithm specialised for nc <= 64 columns (one per lane) with a register
// accessor (RegCostF32, HaaRegCost): `remaining` membership is a scalar 64-bit mask
// (turned into a lane predicate by inverse-ballot, so no per-lane compare), the row read
// is a uniform branch plus one indexed move, and column removal is scalar mask work.
// Identical decisions to lsa_solve_wave<1> (same keys, same tie rule, same float64
// operation order); ~30 vector instructions per augmenting-path step instead of ~42.
// kCount: also count the augmenting-path steps (iterations of scipy's inner loop, the
// figure ora_lsa_iterations reports) into *steps -- an instrumentation instance for the
// LSA efficiency figure; the product instances compile it out.
// a double from its two 32-bit halves as one register pair (no 64-bit OR)
typedef uint32_t lsa_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double dbl_of(uint32_t lo, uint32_t hi) { return __builtin_bit_cast(double, lsa_u32x2{lo, hi}); }

// index of the lowest set bit of a wave-uniform 64-bit mask as one s_ff1_i32_b64, defined for
// every input (-1 for an empty mask, whose low six bits read lane 63); __builtin_ctzll(0) would
// be poison the optimizer may reason from
__device__ __forceinline__ int sff1(uint64_t x) {
    int r;
    asm("s_ff1_i32_b64 %0, %1" : "=s"(r) : "s"(x));
    return r;
}

// index of the highest set bit of a wave-uniform 64-bit mask (s_flbit counts from the MSB;
// -1 for an empty mask)
__device__ __forceinline__ int sfl1(uint64_t x) {
    int r;
    asm("s_flbit_i32_b64 %0, %1" : "=s"(r) : "s"(x));
    return 63 - r;  // an empty mask: 64, lane 0 once masked
}

#ifndef ASG_LSA_COLAT
#define ASG_LSA_COLAT 0
#endif
#if ASG_LSA_COLAT
// lsa_solve_reg64 with scipy's `remaining` list held as it is -- lane `it` holds the column at
// position it (colat), the swap-with-last removal one readlane + one writelane -- instead of
// each column's position.  The tie rule then needs no reduction: the positions whose column is
// a candidate are one ballot (a per-lane shift of the uniform candidate mask), and the largest
// (an unassigned candidate exists) or smallest position is one s_flbit / s_ff1 of it; the
// assigned columns are a scalar mask.  Same decisions as lsa_solve_reg64.
template <class Acc, bool kCount = false>
__device__ int lsa_solve_reg64_colat(const Acc &acc, int nr, int nc, int (&col4row)[1], int *steps) {
    int nsteps = 0;
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t colmask = nc >= 64 ? ~0ull : ((1ull << nc) - 1ull);
    const float kOutF = __builtin_bit_cast(float, 0x7fc00000u);
    double v = 0.0, u = 0.0;
    int r4c = -1, path = -1, c4r = -1;
    uint64_t asg = 0;  // columns assigned to a row (r4c != -1)
    for (int cur = 0; cur < nr; ++cur) {
        double spc = __builtin_inf();
        int colat = (lane < nc) ? (nc - 1 - lane) : 0;  // remaining[it] = nc - it - 1
        uint64_t rem = colmask;                          // columns still in `remaining`
        uint64_t posmask = colmask;  // positions 0 .. nrem - 1 are `remaining`; past them stale copies
        int nrem = nc;
        double minv = 0.0;
        int i = cur, jsel, ncand;
        uint32_t lowest_hi;
        do {
            i = __builtin_amdgcn_readfirstlane(i);
            if (kCount) ++nsteps;
            const double ui = __builtin_bit_cast(double, ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(
                                                              (int)(uint32_t)__builtin_bit_cast(uint64_t, u), i)) |
                                                             ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(
                                                                  (int)(uint32_t)(__builtin_bit_cast(uint64_t, u) >> 32), i)
                                                              << 32));
            const bool remb = __builtin_amdgcn_inverse_ballot_w64(rem);
            const double r = ((minv + acc.col(i)) - ui) - v;
            const bool upd = remb && r < spc;
            spc = upd ? r : spc;
            path = upd ? i : path;
            const float key = remb ? (float)spc : kOutF;
            const float kmin = wave_min_f32_nonan(key);
            const uint64_t cm = __ballot(key == kmin);
            asm("s_bcnt1_i32_b64 %0, %1" : "=s"(ncand) : "s"(cm));
            const uint64_t sb = __builtin_bit_cast(uint64_t, spc);
            jsel = sff1(cm);
            uint32_t lowest_lo = __builtin_amdgcn_readlane((int)(uint32_t)sb, jsel);
            lowest_hi = __builtin_amdgcn_readlane((int)(uint32_t)(sb >> 32), jsel);
            // the first candidate's position (the selection when it is the only one); the tie
            // branch below overrides it -- no else branch for the structurizer to flag
            int psel = sff1(__ballot(colat == jsel) & posmask);
            if (ncand != 1) {
                double lowest0 = dbl_of(lowest_lo, lowest_hi);
                uint64_t cand = cm;
                if ((__ballot(spc != lowest0) & cm) != 0) {
                    const double lo = remb ? spc : __builtin_inf();
                    const uint64_t lb = __builtin_bit_cast(uint64_t, wave_min_f64(lo));
                    lowest_lo = __builtin_amdgcn_readfirstlane((uint32_t)lb);
                    lowest_hi = __builtin_amdgcn_readfirstlane((uint32_t)(lb >> 32));
                    lowest0 = dbl_of(lowest_lo, lowest_hi);
                    cand = __ballot(spc == lowest0) & rem;
                }
                // scipy's tie rule: the unassigned candidate of largest position, else the
                // candidate of smallest position
                const uint64_t un = cand & ~asg;
                const uint64_t S = un ? un : cand;
                const uint64_t at = __ballot(((S >> colat) & 1ull) != 0) & posmask;
                psel = un ? sfl1(at) : sff1(at);
                jsel = __builtin_amdgcn_readlane(colat, psel) & 63;
                if (ncand == 0) lowest_hi = 0x7ff00000u;
            }
            // remaining[psel] = remaining[--num_remaining]
            const int moved = __builtin_amdgcn_readlane(colat, nrem - 1);
            // the lane select in M0 (an SGPR data operand takes gfx9's one constant-bus read)
            asm("v_writelane_b32 %0, %1, m0" : "+v"(colat) : "s"(moved), "{m0}"(psel & 63));
            asm("s_bitset0_b64 %0, %1" : "+s"(rem) : "s"(jsel) : "scc");
            --nrem;
            asm("s_bitset0_b64 %0, %1" : "+s"(posmask) : "s"(nrem) : "scc");
            minv = dbl_of(lowest_lo, lowest_hi);
            i = __builtin_amdgcn_readlane(r4c, jsel);
        } while (__builtin_elementwise_min((uint32_t)(i + 1), lowest_hi ^ 0x7ff00000u) != 0u);
        if (ncand == 0) return ASG_E_LSA_INVALID;
        if (lowest_hi == 0x7ff00000u) return ASG_E_LSA_INFEASIBLE;
        const int sink = jsel;
        asm("s_bitset1_b64 %0, %1" : "+s"(asg) : "s"(sink) : "scc");  // the sink joins the assigned columns
        const int jm = c4r;
        const double spc_j = __shfl(spc, jm & 63, kWave);
        const bool sc_j = jm >= 0 && ((rem >> (jm & 63)) & 1ull) == 0;
        if (lane < nr) {
            if (lane == cur) u += minv;
            else if (sc_j) u += minv - spc_j;
        }
        if (lane < nc && ((rem >> lane) & 1ull) == 0) v -= minv - spc;
        int j = sink;
        while (true) {
            const int pi = __builtin_amdgcn_readlane(path, j);
            r4c = (lane == j) ? pi : r4c;
            const int t = __builtin_amdgcn_readlane(c4r, pi);
            c4r = (lane == pi) ? j : c4r;
            j = t;
            if (pi == cur) break;
        }
    }
    col4row[0] = c4r;
    if (kCount) *steps = nsteps;
    return ASG_OK;
}
#endif

template <class Acc, bool kCount = false>
__device__ int lsa_solve_reg64(const Acc &acc, int nr, int nc, int (&col4row)[1], int *steps = nullptr) {
#ifdef ASG_LSA_GENERIC_REG
    return lsa_solve_wave<1>(acc, nr, nc, col4row);
#elif ASG_LSA_COLAT
    return lsa_solve_reg64_colat<Acc, kCount>(acc, nr, nc, col4row, steps);
#else
    int nsteps = 0;
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t colmask = nc >= 64 ? ~0ull : ((1ull << nc) - 1ull);  // lanes that hold a column
#ifndef ASG_LSA_NAN_KEYS
#define ASG_LSA_NAN_KEYS 1
#endif
    // keys of columns out of `remaining`: a quiet NaN is never equal to the minimum (and
    // v_min_f32 skips it), so the candidate ballot needs no "& rem"
    const float kOutF = ASG_LSA_NAN_KEYS ? __builtin_bit_cast(float, 0x7fc00000u) : __builtin_inff();
    double v = 0.0, u = 0.0;
    int r4c = -1, path = -1, c4r = -1;
    for (int cur = 0; cur < nr; ++cur) {
        double spc = __builtin_inf();
        int pos = (lane < nc) ? (nc - 1 - lane) : -1;  // remaining[it] = nc - it - 1
        uint64_t rem = colmask;                         // columns still in `remaining`
        int nrem = nc;
        double minv = 0.0;
        int i = cur, jsel, ncand;
        uint32_t lowest_hi;
        // Scalar work per step is the issue bound here (one scalar unit serves the CU's four
        // SIMDs): the common single-candidate step is branch-light, the loop has one exit
        // (no early returns the control-flow structurizer would turn into flag chains), the
        // candidate count is one s_bcnt1.
        do {
            i = __builtin_amdgcn_readfirstlane(i);
            if (kCount) ++nsteps;
            const double ui = __builtin_bit_cast(double, ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(
                                                              (int)(uint32_t)__builtin_bit_cast(uint64_t, u), i)) |
                                                             ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(
                                                                  (int)(uint32_t)(__builtin_bit_cast(uint64_t, u) >> 32), i)
                                                              << 32));
            const bool remb = __builtin_amdgcn_inverse_ballot_w64(rem);
            const double r = ((minv + acc.col(i)) - ui) - v;
            const bool upd = remb && r < spc;
            spc = upd ? r : spc;
            path = upd ? i : path;
            const float key = remb ? (float)spc : kOutF;
            const float kmin = wave_min_f32_nonan(key);
            const uint64_t cm = ASG_LSA_NAN_KEYS ? __ballot(key == kmin) : (__ballot(key == kmin) & rem);
            asm("s_bcnt1_i32_b64 %0, %1" : "=s"(ncand) : "s"(cm));
            const uint64_t sb = __builtin_bit_cast(uint64_t, spc);
            jsel = sff1(cm);  // the first candidate: the selection when it is the only one (ncand 0: -1)
            uint32_t lowest_lo = __builtin_amdgcn_readlane((int)(uint32_t)sb, jsel);
            lowest_hi = __builtin_amdgcn_readlane((int)(uint32_t)(sb >> 32), jsel);
            int psel = __builtin_amdgcn_readlane(pos, jsel);
            if (ncand != 1) {
                // equal keys: exact float64 ties (checked against the first candidate) or,
                // rarely, distinct doubles rounding to one float (exact minimum first).  No
                // candidate (ncand 0) only if a cost turned NaN during the solve (e.g. a NaN
                // T_trans entry under HAA): scipy's "invalid numeric entries" -- the step
                // then ends the loop as infeasible and is reported as invalid below
                double lowest0 = dbl_of(lowest_lo, lowest_hi);
                uint64_t cand = cm;
                if ((__ballot(spc != lowest0) & cm) != 0) {
                    const double lo = remb ? spc : __builtin_inf();
                    const uint64_t lb = __builtin_bit_cast(uint64_t, wave_min_f64(lo));
                    lowest_lo = __builtin_amdgcn_readfirstlane((uint32_t)lb);
                    lowest_hi = __builtin_amdgcn_readfirstlane((uint32_t)(lb >> 32));
                    lowest0 = dbl_of(lowest_lo, lowest_hi);
                    cand = __ballot(spc == lowest0) & rem;
                }
                // scipy's tie rule: unassigned 2^31 | pos (largest position), else 2^30 - pos
                // (smallest position), max-reduced
                const bool cb = __builtin_amdgcn_inverse_ballot_w64(cand);
                const uint32_t k = (r4c == -1) ? (0x80000000u | (uint32_t)pos) : ((1u << 30) - (uint32_t)pos);
                const uint32_t tk = wave_max_u32_bcast(cb ? k : 0u);
                psel = (tk >> 31) ? (int)(tk & 0x7fffffffu) : (int)((1u << 30) - tk);
                jsel = sff1(__ballot(pos == psel) & rem) & 63;  // positions are distinct
                if (ncand == 0) lowest_hi = 0x7ff00000u;
            }
            // remaining[index] = remaining[--num_remaining]
            const int last = nrem - 1;
            // (a removed column keeps a stale position: every read of pos is masked by rem)
            pos = pos == last ? psel : pos;
            asm("s_bitset0_b64 %0, %1" : "+s"(rem) : "s"(jsel) : "scc");  // rem &= ~(1 << jsel), one instruction
            --nrem;
            minv = dbl_of(lowest_lo, lowest_hi);
            i = __builtin_amdgcn_readlane(r4c, jsel);
            // continue while the column is assigned (owner != -1) and scipy's minVal is not
            // INFINITY (lowest is never NaN: a NaN key is no candidate and the exact minimum
            // skips NaN, so the high word decides): one unsigned min, one compare
        } while (__builtin_elementwise_min((uint32_t)(i + 1), lowest_hi ^ 0x7ff00000u) != 0u);
        if (ncand == 0) return ASG_E_LSA_INVALID;
        if (lowest_hi == 0x7ff00000u) return ASG_E_LSA_INFEASIBLE;
        const int sink = jsel;
        // dual update: u[cur] += minv; u[r] += minv - spc[col4row[r]] for the other visited
        // rows (row r != cur was visited iff its column was scanned); v[j] -= minv - spc[j]
        // for the scanned columns (matrix columns no longer in `remaining`)
        const int jm = c4r;
        const double spc_j = __shfl(spc, jm & 63, kWave);
        const bool sc_j = jm >= 0 && ((rem >> (jm & 63)) & 1ull) == 0;
        if (lane < nr) {
            if (lane == cur) u += minv;
            else if (sc_j) u += minv - spc_j;
        }
        if (lane < nc && ((rem >> lane) & 1ull) == 0) v -= minv - spc;
        // augment along path back to cur
        int j = sink;
        while (true) {
            const int pi = __builtin_amdgcn_readlane(path, j);
            r4c = (lane == j) ? pi : r4c;
            const int t = __builtin_amdgcn_readlane(c4r, pi);
            c4r = (lane == pi) ? j : c4r;
            j = t;
            if (pi == cur) break;
        }
    }
    col4row[0] = c4r;
    if (kCount) *steps = nsteps;
    return ASG_OK;
#endif
}

// ------------------------------------------------------------------------------------
// Certified fast path for square register-resident problems (nr == nc <= 64).
//
// scipy's algorithm starts every row's Dijkstra from u = v = 0 and an empty matching; on
// SAP Q-values (one shared task profile, small per-agent terms) that costs ~1,400
// augmenting-path steps per 64 x 64 problem.  Here the SAME shortest-augmenting-path step
// runs from a row + column reduction instead (u_i = min_j c_ij, v_j = min_i (c_ij - u_i): dual
// feasible; each row keeps a column whose minimum it holds: complementary slack), so only the
// rows the reduction leaves free are augmented: ~0.4x the steps on SAP-like matrices
// (tools/lsa_fastpath_sim.py).  Ties among equal path costs go to the lowest lane:
// any shortest-path choice yields AN optimal assignment.
//
// Which optimum scipy returns only matters when the optimum is not unique, so the result is
// used only under a uniqueness certificate computed from the final duals (u, v), with
// S = max|c| + max|u| + max|v| and reduced costs rc_ij = (c_ij - u_i) - v_j:
//   (1) rc_ij >= -S 2^-40 everywhere and rc <= S 2^-40 on the matching (dual feasibility and
//       complementary slackness up to rounding: each dual carries at most ~2 roundings per
//       augmentation, < S 2^-46 after 64 of them);
//   (2) the graph "row i -> row owning column j" over the near-tight edges (rc_ij <= S 2^-30,
//       j not i's column) is acyclic (peeled source by source).
// Every other assignment differs from this one by alternating cycles, each of which
// contains a non-tight edge by (2), so its cost exceeds this one's by more than
// S 2^-30 - 128 S 2^-40 > S 2^-31 (exact arithmetic on the float64 working matrix).  scipy's
// float64 run makes the same kind of roundings (< S 2^-46 per reduced cost), so its result is
// optimal to within 64 such errors (< S 2^-39) -- 2^8 below the margin: it is this
// assignment.  When (1) or (2) fails (exact or near ties, NaN) the caller runs the
// scipy-exact solver from scratch.
// Returns ASG_OK (col4row set), or kLsaUncertified.  `slot`: 64 uint64 of LDS scratch for
// this wave.
//
// Warm start (kWarm, `vwarm` = this lane's column dual from an earlier call, e.g. the previous
// step's selection of the same env): the row duals start as u_k = min_j (c_kj - vwarm_j), and
// the usual column reduction and claims follow (see the dual start below).  The result is the
// same: whatever duals the search starts from, the assignment is used only under the
// certificate below, else the scipy-exact solver runs.  Non-finite warm duals (the first call)
// take the cold start.  `vout` (optional) receives the final column duals, shifted so their
// minimum is 0.
constexpr int kLsaUncertified = 1;

__device__ __forceinline__ double lane_dbl(double x, int src) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    return dbl_of((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, src),
                  (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), src));
}

template <class Acc, bool kCount = false, bool kWarm = false>
__device__ int lsa_fast_reg64(const Acc &acc, int n, int (&col4row)[1], int *steps, uint64_t *slot, double vwarm = 0.0,
                              double *vout = nullptr) {
    int nsteps = 0;
    const int lane = threadIdx.x & (kWave - 1);
    const bool live = lane < n;
    const uint64_t colmask = n >= 64 ? ~0ull : ((1ull << n) - 1ull);
    const float kOutF = __builtin_bit_cast(float, 0x7fc00000u);
    int r4c = -1, c4r = -1;
    double v = 0.0, u = 0.0;
    float amax = 0.0f;
    // the dual start: u, then the column reduction v_j = min_k (c_kj - u_k) with each row keeping
    // the lowest column whose minimum it holds.  Cold: u_k = min_j c_kj (float32: exact).  Warm
    // (kWarm, finite vwarm on every live lane): u_k = min_j (c_kj - vwarm_j) in float64 -- the
    // previous call's column duals carry over into the row duals, and the column reduction then
    // fits v to this problem (REDA's own Q sequence: 0.50x the cold start's augmenting-path
    // steps in the host model, 0.36x on the GRU agent's at eps 0.05; taking the previous v as the
    // start itself, without the column reduction, took 1.04x / 0.72x)
    double vmin = __builtin_inf();
    int imin = 0;
    bool warm = false;
    if constexpr (kWarm) warm = __ballot(live && !(__builtin_fabs(vwarm) < __builtin_inf())) == 0;
    if constexpr (kWarm) {
        // one rolled loop for both starts (the row through the indexed read): two unrolled copies
        // had overflowed the SGPR file (~200 spilled)
        const double vw = (live && warm) ? vwarm : 0.0;
#pragma unroll 1
        for (int k = 0; k < 64; ++k) {
            if (k < n) {
                const float x = acc.col(k);
                double uk;
                if (warm) {
                    const double d = live ? (double)x - vw : __builtin_inf();
                    const float key = (float)d;
                    const float kmin = wave_min_f32_nonan(live ? key : __builtin_inff());
                    const uint64_t cm = __ballot(key == kmin);
                    if (cm == 0) {  // every entry of the row NaN: the exact solver reports it
                        if (kCount) *steps = nsteps;
                        return kLsaUncertified;
                    }
                    uk = lane_dbl(d, sff1(cm));
                    if ((__ballot(d != uk) & cm) != 0) {  // distinct doubles behind one float key
                        const uint64_t lb =
                            __builtin_bit_cast(uint64_t, wave_min_f64(((cm >> lane) & 1ull) ? d : __builtin_inf()));
                        uk = dbl_of(__builtin_amdgcn_readfirstlane((uint32_t)lb),
                                    __builtin_amdgcn_readfirstlane((uint32_t)(lb >> 32)));
                    }
                } else {
                    uk = (double)wave_min_f32_nonan(live ? x : __builtin_inff());
                }
                u = lane == k ? uk : u;
                const double r = (double)x - uk;
                const bool t = r < vmin;
                vmin = t ? r : vmin;
                imin = t ? k : imin;
                amax = __builtin_fmaxf(amax, __builtin_fabsf(x));
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < 64; ++k) {
            if (k < n) {
                const float x = k < 32 ? acc.lo[k] : acc.hi[k - 32];
                const float uk = wave_min_f32_nonan(live ? x : __builtin_inff());
                u = lane == k ? (double)uk : u;
                const double r = (double)x - (double)uk;
                const bool t = r < vmin;
                vmin = t ? r : vmin;
                imin = t ? k : imin;
                amax = __builtin_fmaxf(amax, __builtin_fabsf(x));
            }
        }
    }
    // (float32 row minima are exact; the column reduction's float64 differences are rounded once,
    // relative 2^-53, far inside the certificate's S 2^-40 slack -- not exact when the operands'
    // exponents differ by more than ~29 bits; dual feasibility is re-checked by the certificate)
    // each row keeps one of the columns whose minimum it holds (the lowest: any keeps
    // complementary slackness, rc = 0 there): one LDS minimum per column
    uint32_t *slot32 = reinterpret_cast<uint32_t *>(slot);
    slot32[lane] = 0xffffffffu;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (live) atomicMin(&slot32[imin], (uint32_t)lane);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t won = slot32[imin], mine = slot32[lane];
    r4c = (live && won == (uint32_t)lane) ? imin : -1;
    c4r = (live && mine != 0xffffffffu) ? (int)mine : -1;
    v = live ? vmin : 0.0;
    int path = -1;
    uint64_t freerows = __ballot(live && c4r < 0);
    int ncand = 1;
    uint32_t lowest_hi = 0;
    while (freerows != 0) {
        const int cur = sff1(freerows);
        asm("s_bitset0_b64 %0, %1" : "+s"(freerows) : "s"(cur) : "scc");
        double spc = __builtin_inf();
        uint64_t rem = colmask;
        // the distance of the last scanned column (minv), kept as its two words
        uint32_t lowest_lo = 0;
        lowest_hi = 0;
        const uint64_t freec = __ballot(live && r4c < 0);  // unassigned columns: a tie among them ends the search
        int i = cur, jsel;
        do {
            i = __builtin_amdgcn_readfirstlane(i);
            if (kCount) ++nsteps;
            const double minv = dbl_of(lowest_lo, lowest_hi);
            const double ui = lane_dbl(u, i);
            const bool remb = __builtin_amdgcn_inverse_ballot_w64(rem);
            const double r = ((minv + acc.col(i)) - ui) - v;
            const bool upd = remb && r < spc;
            spc = upd ? r : spc;
            path = upd ? i : path;
            // columns still at exactly the current distance (zero reduced costs, two thirds of
            // the steps on SAP Q): one of them is next -- every remaining distance is >= minv --
            // so no reduction; an unassigned one ends the search
            const uint64_t tie = __builtin_amdgcn_ballot_w64(spc == minv) & rem;  // compare straight into an SGPR pair
            if (tie != 0) {
                const uint64_t tf = tie & freec;
                jsel = sff1(tf != 0 ? tf : tie);
                ncand = 1;
            } else {
                const float fkey = remb ? (float)spc : kOutF;
                const float kmin = wave_min_f32_nonan(fkey);
                const uint64_t cm = __ballot(fkey == kmin);
                asm("s_bcnt1_i32_b64 %0, %1" : "=s"(ncand) : "s"(cm));
                const uint64_t sb = __builtin_bit_cast(uint64_t, spc);
                jsel = sff1(cm);
                lowest_lo = __builtin_amdgcn_readlane((int)(uint32_t)sb, jsel);
                lowest_hi = __builtin_amdgcn_readlane((int)(uint32_t)(sb >> 32), jsel);
                if (ncand != 1) {
                    // equal keys: any column at the exact float64 minimum is a shortest-path choice
                    if ((__ballot(spc != dbl_of(lowest_lo, lowest_hi)) & cm) != 0) {
                        const uint64_t lb = __builtin_bit_cast(uint64_t, wave_min_f64(remb ? spc : __builtin_inf()));
                        lowest_lo = __builtin_amdgcn_readfirstlane((uint32_t)lb);
                        lowest_hi = __builtin_amdgcn_readfirstlane((uint32_t)(lb >> 32));
                        jsel = sff1(__ballot(spc == dbl_of(lowest_lo, lowest_hi)) & rem) & 63;
                    }
                    if (ncand == 0) lowest_hi = 0x7ff00000u;  // NaN mid-solve: leave, uncertified
                }
            }
            asm("s_bitset0_b64 %0, %1" : "+s"(rem) : "s"(jsel) : "scc");
            i = __builtin_amdgcn_readlane(r4c, jsel);
        } while (__builtin_elementwise_min((uint32_t)(i + 1), lowest_hi ^ 0x7ff00000u) != 0u);
        if (ncand == 0 || lowest_hi == 0x7ff00000u) {
            if (kCount) *steps = nsteps;
            return kLsaUncertified;
        }
        const int sink = jsel;
        const double minv = dbl_of(lowest_lo, lowest_hi);
        // scipy's dual update (u[cur] += minv; visited rows u[r] += minv - spc[col4row[r]];
        // scanned columns v[j] -= minv - spc[j]) and augmentation, as lsa_solve_reg64
        const int jm = c4r;
        const double spc_j = __shfl(spc, jm & 63, kWave);
        const bool sc_j = jm >= 0 && ((rem >> (jm & 63)) & 1ull) == 0;
        if (live) {
            if (lane == cur) u += minv;
            else if (sc_j) u += minv - spc_j;
        }
        if (live && ((rem >> lane) & 1ull) == 0) v -= minv - spc;
        int j = sink;
        while (true) {
            const int pi = __builtin_amdgcn_readlane(path, j);
            r4c = (lane == j) ? pi : r4c;
            const int t = __builtin_amdgcn_readlane(c4r, pi);
            c4r = (lane == pi) ? j : c4r;
            j = t;
            if (pi == cur) break;
        }
    }
    if (kCount) *steps = nsteps;
    if (kWarm && vout) {
        // the next call's warm start, shifted to a zero minimum (bounded S across calls)
        const double vm = wave_min_f64(live ? v : __builtin_inf());
        *vout = v - vm;
    }
#ifdef ASG_LSA_FAST_NOCERT  // timing experiments only: what the certificate costs (wrong on ties)
    col4row[0] = c4r;
    return ASG_OK;
#endif
    // the certificate
    const float am = wave_max_f32_nonan(amax);
    const double ua = wave_allreduce(live ? __builtin_fabs(u) : 0.0, [](double a, double b) { return fmax(a, b); });
    const double va = wave_allreduce(live ? __builtin_fabs(v) : 0.0, [](double a, double b) { return fmax(a, b); });
    const double S = ((double)am + ua) + va;
    if (!(S < __builtin_inf())) return kLsaUncertified;
    const double tight = S * 0x1p-30, slack = S * 0x1p-40;
    // lane j (column j, matched to row r4c) collects tin: the rows i != r4c whose edge (i, j) is
    // near-tight -- the in-edges of node r4c in the graph "row i -> row r4c(j)" -- from its own
    // register column, four rows at a time
    uint64_t tin = 0;
    bool bad = false;
    for (int k0 = 0; k0 < n; k0 += 4) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {  // four independent rows per iteration
            const int k = __builtin_amdgcn_readfirstlane(k0 + kk);
            const double rc = ((double)acc.col(k) - lane_dbl(u, k)) - v;
            const bool row = live && k < n;
            bad |= (row && !(rc >= -slack)) | (k == r4c && !(rc <= slack));
            tin |= (row && k != r4c && rc <= tight) ? 1ull << k : 0ull;
        }
    }
    if (wave_or_i32(bad)) return kLsaUncertified;
    // peel the sources (alive rows with no near-tight in-edge from an alive row) until none is
    // left (acyclic) or none can go (a cycle: another optimum within S 2^-30).  Lane j speaks for
    // row r4c; lane i learns whether its own row left through its column c4r.
    uint64_t A = colmask;
    while (A != 0) {
        const uint64_t srcc = __ballot(live && ((A >> (r4c & 63)) & 1ull) != 0 && (tin & A) == 0);
        const uint64_t gone = __ballot(live && ((srcc >> (c4r & 63)) & 1ull) != 0);
        if (gone == 0) return kLsaUncertified;
        A &= ~gone;
    }
    col4row[0] = c4r;
    return ASG_OK;
}

// Stage C (input [nr0][nc0], strides in elements) into dst as scipy's working matrix:
// transposed when nr0 > nc0, negated for maximize.  Returns ASG_E_LSA_INVALID (wave
// uniform) when an entry is NaN or -inf after the sign flip.
template <typename IT, typename CT>
__device__ int lsa_stage_wave(const IT *C, int64_t rs, int64_t cs, int nr0, int nc0,
                              bool maximize, CT *dst) {
    const int lane = threadIdx.x & (kWave - 1);
    const bool tr = nc0 < nr0;
    const int nc = tr ? nr0 : nc0;
    int bad = 0;
    for (int idx = lane; idx < nr0 * nc0; idx += kWave) {
        const int r = idx / nc0, c = idx - r * nc0;
        CT x = (CT)C[r * rs + c * cs];
        if (maximize) x = -x;
        bad |= (x != x) || (x == -(CT)__builtin_inf());
        if (tr) dst[(size_t)c * nc + r] = x; else dst[(size_t)r * nc + c] = x;
    }
    wave_sync();
    return wave_or_i32(bad) ? ASG_E_LSA_INVALID : ASG_OK;
}

// scipy's output convention from the working solution: (arange(nr), col4row) or, when
// transposed, (col4row[argsort(col4row)], argsort(col4row)).  `mark` is LDS scratch of
// nr0 ints (only used when transposed).
template <int CPL>
__device__ void lsa_emit_wave(const int (&col4row)[CPL], int nr0, int nc0, int *mark, int64_t *row_out,
                              int64_t *col_out, float *colf_out) {
    const int lane = threadIdx.x & (kWave - 1);
    if (nc0 >= nr0) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int r = lane + kWave * c;
            if (r < nr0) {
                if (row_out) row_out[r] = r;
                if (col_out) col_out[r] = col4row[c];
                if (colf_out) colf_out[r] = (float)col4row[c];
            }
        }
        return;
    }
    // transposed: working rows are original columns (nc0 of them), col4row is the
    // original row matched to each original column; emit sorted by original row
    for (int r = lane; r < nr0; r += kWave) mark[r] = -1;
    wave_sync();
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
        const int oc = lane + kWave * c;
        if (oc < nc0) mark[col4row[c]] = oc;
    }
    wave_sync();
    int base = 0;
    for (int r0 = 0; r0 < nr0; r0 += kWave) {
        const int r = r0 + lane;
        const bool has = r < nr0 && mark[r] >= 0;
        const uint64_t bal = __ballot(has);
        const int off = __popcll(bal & ((1ull << lane) - 1ull));
        if (has) {
            if (row_out) row_out[base + off] = r;
            if (col_out) col_out[base + off] = mark[r];
            if (colf_out) colf_out[base + off] = (float)mark[r];
        }
        base += __popcll(bal);
    }
}

}  // namespace asg
