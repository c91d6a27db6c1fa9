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

// Scratch in LDS for one problem: u[nr] (f64), col4row[nr], row4col[nc], path[nc] (i32)
struct LsaScratch {
    double *u;
    int *col4row;
    int *row4col;
    int *path;
};

// Row-major cost matrix in LDS (already transposed / sign-flipped)
template <typename CT>
struct DenseCost {
    const CT *c;
    int nc;
    __device__ double operator()(int i, int j) const { return (double)c[(size_t)i * nc + j]; }
};

// Solve on the working matrix acc(i, j), i < nr <= nc <= 64*CPL (scipy's orientation).
// Returns 0 or ASG_E_LSA_INFEASIBLE; s.col4row holds the assignment.
// All 64 lanes of the wave must call it with identical arguments.
template <int CPL, class Acc>
__device__ int lsa_solve_wave(const Acc &acc, int nr, int nc, LsaScratch s) {
    const int lane = threadIdx.x & (kWave - 1);
    for (int r = lane; r < nr; r += kWave) {
        s.u[r] = 0.0;
        s.col4row[r] = -1;
    }
    double v[CPL];
    int r4c[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
        const int j = lane + kWave * c;
        v[c] = 0.0;
        r4c[c] = -1;
        if (j < nc) {
            s.row4col[j] = -1;
            s.path[j] = -1;
        }
    }
    wave_sync();

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
            const double ui = s.u[i];
            double lo = __builtin_inf();
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int j = lane + kWave * c;
                if (pos[c] >= 0) {
                    const double r = ((minv + acc(i, j)) - ui) - v[c];
                    if (r < spc[c]) {
                        spc[c] = r;
                        s.path[j] = i;
                    }
                    lo = fmin(lo, spc[c]);
                }
            }
            const double lowest = wave_min_f64(lo);
            if (lowest == __builtin_inf()) return ASG_E_LSA_INFEASIBLE;  // uniform branch
            // packed selection key, reduced with max:
            //   bit 63      : candidate is unassigned
            //   bits 62..32 : unassigned ? pos : (2^30 - pos)   (largest pos vs smallest pos)
            //   bits 31..0  : column index
            uint64_t key = 0;
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int j = lane + kWave * c;
                if (pos[c] >= 0 && spc[c] == lowest) {
                    const bool un = r4c[c] == -1;
                    const uint64_t k = un ? ((1ull << 63) | ((uint64_t)pos[c] << 32) | (uint32_t)j)
                                          : (((uint64_t)((1u << 30) - (uint32_t)pos[c]) << 32) | (uint32_t)j);
                    key = k > key ? k : key;
                }
            }
            key = wave_max_u64(key);
            const int jsel = (int)(uint32_t)key;
            const int last = nrem - 1;
            int psel = -1;
#pragma unroll
            for (int c = 0; c < CPL; ++c)
                if (lane + kWave * c == jsel) psel = pos[c];
            psel = wave_max_i32(psel);
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
            const int owner = s.row4col[jsel];
            if (owner == -1) sink = jsel; else i = owner;
        }
        // dual update: u[cur] += minv; u[row4col[j]] += minv - spc[j] for the other
        // rows of the tree (one per scanned assigned column); v[j] -= minv - spc[j]
        if (lane == 0) s.u[cur] += minv;
        wave_sync();
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int j = lane + kWave * c;
            if (sc[c]) {
                const double d = minv - spc[c];
                if (j != sink) s.u[r4c[c]] += d;
                v[c] -= d;
            }
        }
        wave_sync();
        // augment along path back to cur
        if (lane == 0) {
            int j = sink;
            while (true) {
                const int pi = s.path[j];
                s.row4col[j] = pi;
                const int t = s.col4row[pi];
                s.col4row[pi] = j;
                j = t;
                if (pi == cur) break;
            }
        }
        wave_sync();
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int j = lane + kWave * c;
            if (j < nc) r4c[c] = s.row4col[j];
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
__device__ inline void lsa_emit_wave(const int *col4row, int nr0, int nc0, int *mark,
                                     int64_t *row_out, int64_t *col_out, float *colf_out) {
    const int lane = threadIdx.x & (kWave - 1);
    if (nc0 >= nr0) {
        for (int r = lane; r < nr0; r += kWave) {
            if (row_out) row_out[r] = r;
            if (col_out) col_out[r] = col4row[r];
            if (colf_out) colf_out[r] = (float)col4row[r];
        }
        return;
    }
    // transposed: working rows are original columns (nc0 of them), col4row[c] is the
    // original row matched to original column c; emit sorted by original row
    for (int r = lane; r < nr0; r += kWave) mark[r] = -1;
    wave_sync();
    for (int c = lane; c < nc0; c += kWave) mark[col4row[c]] = c;
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
