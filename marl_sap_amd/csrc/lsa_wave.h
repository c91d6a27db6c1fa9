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
// The cost matrix lives in LDS (or global memory for large problems) already
// transposed (nr <= nc) and sign-flipped for maximize, as scipy does before solving.
#pragma once
#include "asg_device.h"

namespace asg {

// Row-major cost matrix in LDS (already transposed / sign-flipped)
template <typename CT>
struct DenseCost {
    const CT *c;
    int nc;
    __device__ double operator()(int i, int j) const { return (double)c[(size_t)i * nc + j]; }
};

// Solve on the working matrix acc(i, j), i < nr <= nc <= 64*CPL (scipy's orientation).
// All per-row and per-column state lives in registers, distributed over the lanes
// (column j / row r in lane j%64, slot j/64); only the cost matrix is in memory.  The
// per-iteration reductions are VALU butterflies (DPP + permlane swaps) and the uniform
// reads are v_readlane, so the serial augmenting-path loop has no LDS round trip except
// the cost-row read.  Returns 0 or ASG_E_LSA_INFEASIBLE; col4row[c] holds the column
// assigned to row lane + 64c.  All 64 lanes must call it with identical arguments.
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
        int pos[CPL];
        bool sc[CPL];
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int j = lane + kWave * c;
            spc[c] = __builtin_inf();
            sc[c] = false;
            pos[c] = (j < nc) ? (nc - 1 - j) : -1;  // remaining[it] = nc - it - 1
        }
        int nrem = nc;
        double minv = 0.0;
        int i = cur, sink = -1;
        while (sink == -1) {
            const double ui = lane_get(u, i);
            double lo = __builtin_inf();
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int j = lane + kWave * c;
                if (pos[c] >= 0) {
                    const double r = ((minv + acc(i, j)) - ui) - v[c];
                    if (r < spc[c]) {
                        spc[c] = r;
                        path[c] = i;
                    }
                    lo = fmin(lo, spc[c]);
                }
            }
            const double lowest = wave_min_f64(lo);
            if (lowest == __builtin_inf()) return ASG_E_LSA_INFEASIBLE;  // uniform branch
            // candidates (remaining columns at the minimum): one ballot per slot.  With a
            // single candidate (the common case for float data) it is the selection;
            // ties fall back to the packed-key reduction below.
            int total = 0, jsel = -1, psel = -1;
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const uint64_t msk = __ballot(pos[c] >= 0 && spc[c] == lowest);
                const int cnt = __popcll(msk);
                if (cnt == 1 && total == 0) {
                    const int src = __builtin_ctzll(msk);
                    jsel = src + kWave * c;
                    psel = __builtin_amdgcn_readlane(pos[c], src);
                }
                total += cnt;
            }
            if (total != 1) {
                // packed selection key, reduced with max:
                //   bit 63      : candidate is unassigned
                //   bits 62..32 : unassigned ? pos : (2^30 - pos)   (largest pos vs smallest pos)
                //   bits 31..0  : column index
                uint64_t key = 0;
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    const int j = lane + kWave * c;
                    if (pos[c] >= 0 && spc[c] == lowest) {
                        const uint64_t k = (r4c[c] == -1)
                                               ? ((1ull << 63) | ((uint64_t)pos[c] << 32) | (uint32_t)j)
                                               : (((uint64_t)((1u << 30) - (uint32_t)pos[c]) << 32) | (uint32_t)j);
                        key = k > key ? k : key;
                    }
                }
                key = wave_max_u64(key);
                const uint32_t khi = __builtin_amdgcn_readfirstlane((uint32_t)(key >> 32));
                jsel = __builtin_amdgcn_readfirstlane((uint32_t)key);
                psel = (khi >> 31) ? (int)(khi & 0x7fffffffu) : (int)((1u << 30) - khi);
            }
            const int last = nrem - 1;
            // remaining[index] = remaining[--num_remaining]
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                if (pos[c] == last) pos[c] = psel;
                if (lane + kWave * c == jsel) {
                    pos[c] = -1;
                    sc[c] = true;
                }
            }
            --nrem;
            minv = lowest;
            const int owner = lane_get(r4c, jsel);
            if (owner == -1) sink = jsel; else i = owner;
        }
        // dual update (scipy: u[cur] += minv; u[r] += minv - spc[col4row[r]] for the
        // other visited rows; v[j] -= minv - spc[j] for the scanned columns).  A row
        // r != cur was visited iff its matched column col4row[r] was scanned.
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int r = lane + kWave * c;
            const int jm = col4row[c];
            // gather (sc, spc) of column jm from its owner lane
            double spc_j = 0.0;
            int sc_j = 0;
#pragma unroll
            for (int c2 = 0; c2 < CPL; ++c2) {
                const double sv = __shfl(spc[c2], jm & 63, kWave);
                const int sb = __shfl((int)sc[c2], jm & 63, kWave);
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
            if (sc[c]) v[c] -= minv - spc[c];
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
