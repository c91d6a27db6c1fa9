// asg_select.hip -- fused epsilon-greedy action selection (gfx950).
//
// EpsilonGreedyActionSelector.select_action (action_selectors/classic_selectors.py:28-54):
// per (env, agent) row of Q-values, with probability epsilon a uniformly random
// AVAILABLE action (Categorical(avail)), otherwise the argmax over available actions
// (masked to -inf; first maximal index, NaN propagating like torch.max).  The reference
// spends a clone, a masked fill, a rand, a Categorical sample, a max and two blends; here
// one pass reads each Q row once (16 lanes x float4 = one 256-B row per lane group, 4
// rows per wave instruction) and writes the int64 action straight into the EpisodeBatch.
#include "asg_device.h"
#include "asg_internal.h"

namespace asg {

// MASK = false: the argmax ignores availability (the filtered selectors' benefit matrix,
// filtered_classic_selectors.py:57-61); exploration still draws over the available tasks
template <bool VEC4, bool MASK>
__global__ void __launch_bounds__(256) eps_greedy_kernel(const float *q, int64_t q0, int64_t q1, int64_t q2,
                                                         const uint8_t *avail, int64_t a0, int64_t a1, int64_t a2,
                                                         int64_t B, int n, int m, float epsilon, uint32_t k0,
                                                         uint32_t k1, uint32_t counter, int64_t row_base,
                                                         int64_t *out, int64_t o0,
                                                         int64_t o1, int *err) {
    const int lane16 = threadIdx.x & 15;
    const int64_t rows = B * n;
    const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const bool live = row < rows;
    const int64_t b = live ? row / n : 0;
    const int i = live ? (int)(row - b * n) : 0;
    const float *qr = q + b * q0 + (int64_t)i * q1;
    const uint8_t *ar = avail + b * a0 + (int64_t)i * a1;
    float best = -__builtin_inff();
    int bj = 0x7fffffff;
    int cnt = 0;
    uint64_t availmask_lo = 0;  // availability bits of this lane's tasks (first 64 chunks)
    int nchunk = 0;
    for (int j0 = lane16 * 4; j0 < m; j0 += 64, ++nchunk) {
        float v[4];
        uint8_t av[4];
        if (VEC4 && j0 + 3 < m) {
            const float4 f = *reinterpret_cast<const float4 *>(qr + j0);
            v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
            const uint32_t w = *reinterpret_cast<const uint32_t *>(ar + j0);
            av[0] = w & 0xff; av[1] = (w >> 8) & 0xff; av[2] = (w >> 16) & 0xff; av[3] = w >> 24;
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const bool in = j0 + c < m;
                v[c] = in ? qr[(j0 + c) * q2] : -__builtin_inff();
                av[c] = in ? ar[(j0 + c) * a2] : 0;
            }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int j = j0 + c;
            if (j >= m) continue;
            const float x = (!MASK || av[c]) ? v[c] : -__builtin_inff();
            if (better(x, j, best, bj)) { best = x; bj = j; }
            cnt += av[c] != 0;
            if (nchunk < 16 && av[c]) availmask_lo |= 1ull << (nchunk * 4 + c);
        }
    }
    // reduce (best, bj) and cnt over the 16-lane group
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) {
        const float ob = __shfl_xor(best, o, 16);
        const int oj = __shfl_xor(bj, o, 16);
        if (better(ob, oj, best, bj)) { best = ob; bj = oj; }
        cnt += __shfl_xor(cnt, o, 16);
    }
    if (bj == 0x7fffffff) bj = 0;
    int action = bj;
    if (epsilon > 0.0f) {
        const int64_t grow = row + row_base;  // global (env, agent) row: shard-invariant draws
        const u32x4 r = philox4x32_10(u32x4{(uint32_t)grow, (uint32_t)(grow >> 32), kCtrSelect, counter}, k0, k1);
        constexpr float k2m24 = 5.9604644775390625e-08f;  // 2^-24
        const bool pick = (float)(r.x >> 8) * k2m24 < epsilon;
        if (pick && cnt > 0) {
            // the target-th available task in index order (Categorical over avail)
            const int target = (int)(((uint64_t)r.y * (uint64_t)cnt) >> 32);
            // per lane count of available tasks, exclusive prefix over the group in
            // index order: task j lives in lane (j / 4) % 16, chunk j / 64
            int found = -1;
            int base = 0;
            for (int ch = 0; ch * 64 < m; ++ch) {
                int mine = 0;
                for (int c = 0; c < 4; ++c) {
                    const int j = ch * 64 + lane16 * 4 + c;
                    if (j < m) {
                        const bool a = ch < 16 ? ((availmask_lo >> (ch * 4 + c)) & 1ull) : (ar[j * a2] != 0);
                        mine += a;
                    }
                }
                int incl = mine;
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    const int y = __shfl_up(incl, o, 16);
                    if (lane16 >= o) incl += y;
                }
                const int excl = base + incl - mine;
                if (found < 0 && target >= excl && target < excl + mine) {
                    int left = target - excl;
                    for (int c = 0; c < 4; ++c) {
                        const int j = ch * 64 + lane16 * 4 + c;
                        if (j < m) {
                            const bool a = ch < 16 ? ((availmask_lo >> (ch * 4 + c)) & 1ull) : (ar[j * a2] != 0);
                            if (a) {
                                if (left == 0) { found = j; break; }
                                --left;
                            }
                        }
                    }
                }
                base += __shfl(incl, 15, 16);
            }
            // exactly one lane of the group found it
#pragma unroll
            for (int o = 8; o >= 1; o >>= 1) found = max(found, __shfl_xor(found, o, 16));
            action = found;
        }
        if (pick && cnt == 0 && lane16 == 0 && live) atomicCAS(err, 0, ASG_E_INVALID_ARG);
    }
    if (live && lane16 == 0) out[b * o0 + (int64_t)i * o1] = action;
}

hipError_t launch_eps_greedy(const float *q, const int64_t qs[3], const uint8_t *avail, const int64_t as[3],
                             int64_t B, int n, int m, float epsilon, uint64_t seed, uint32_t counter,
                             int64_t row_base, int64_t *out, const int64_t os[2], int *err, hipStream_t s,
                             bool mask) {
    const int64_t threads = B * n * 16;
    const int64_t blocks = (threads + 255) / 256;
    const bool v4 = qs[2] == 1 && as[2] == 1 && (reinterpret_cast<uintptr_t>(q) % 16) == 0 &&
                    (reinterpret_cast<uintptr_t>(avail) % 4) == 0 && qs[0] % 4 == 0 && qs[1] % 4 == 0 &&
                    as[0] % 4 == 0 && as[1] % 4 == 0;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ 0x5bd1e995u;
#define EG_(V4, MK)                                                                                             \
    hipLaunchKernelGGL((eps_greedy_kernel<V4, MK>), dim3(blocks), dim3(256), 0, s, q, qs[0], qs[1], qs[2], avail, \
                       as[0], as[1], as[2], B, n, m, epsilon, k0, k1, counter, row_base, out, os[0], os[1], err)
    if (v4) {
        if (mask) EG_(true, true);
        else EG_(true, false);
    } else {
        if (mask) EG_(false, true);
        else EG_(false, false);
    }
#undef EG_
    return hipGetLastError();
}

}  // namespace asg
