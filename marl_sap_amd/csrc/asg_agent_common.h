// asg_agent_common.h -- pieces shared by the f32 / split-bf16 agent kernels (asg_agent.hip)
// and the split-f16 agent + fused rollout kernels (asg_h2.hip): vector types, the hidden
// size, and the epsilon-greedy epilogue fused into every agent kernel.
#pragma once
#include "asg_device.h"
#include "asg_internal.h"

namespace asg {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
constexpr int kHid = 64;  // hidden_dim

__device__ __forceinline__ float comp(const float4 &v, int e) {
    return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
}

// Epilogue of the fused epsilon-greedy selection (asg_select.hip semantics, reference
// action_selectors/classic_selectors.py:28-54): reduce each row's running argmax over its 4
// lanes, then lane q == nt finishes row nt -- the greedy action, or with probability epsilon
// the target-th available task in index order.  best / bj / amask: per-lane partial argmax
// and availability bits of the row's tasks (task 16 c + 4 q + v is bit 4 c + v of lane q's
// mask; GEN: a second word for tasks 256-511).  Writes sel.out and returns the action
// (meaningful on lanes q < NT whose row is ok; row nt = q & 1).
template <bool GEN, int NT, class SA>
__device__ __forceinline__ int select_finish(float (&best)[NT], int (&bj)[NT], const uint64_t (&amask)[NT][2],
                                             const int64_t (&rows)[NT], const bool (&ok)[NT],
                                             const int64_t (&oidx)[NT], int nct, SA &sel, int q) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        auto red = [&](auto swp) {
            const SwapPair pb = swp(__builtin_bit_cast(uint32_t, best[nt]));
            const SwapPair pj = swp((uint32_t)bj[nt]);
            float vb = __builtin_bit_cast(float, pb.a);
            int jb = (int)pj.a;
            if (better(__builtin_bit_cast(float, pb.b), (int)pj.b, vb, jb)) {
                vb = __builtin_bit_cast(float, pb.b);
                jb = (int)pj.b;
            }
            best[nt] = vb;
            bj[nt] = jb;
        };
        red(swap16);
        red(swap32);
    }
    const int nt = NT == 1 ? 0 : (q & 1);
    const int64_t row = rows[nt];
    int action = bj[nt] == 0x7fffffff ? 0 : bj[nt];
    bool explore = false;
    u32x4 rr = u32x4{0u, 0u, 0u, 0u};
    if (sel.epsilon > 0.0f) {
        const int64_t grow = row + sel.row_base;  // global (env, agent) row: shard-invariant draws
        rr = philox4x32_10(u32x4{(uint32_t)grow, (uint32_t)(grow >> 32), kCtrSelect, sel.counter}, sel.k0, sel.k1);
        constexpr float k2m24 = 5.9604644775390625e-08f;
        explore = ok[nt] && q < NT && (float)(rr.x >> 8) * k2m24 < sel.epsilon;
    }
    if (__ballot(explore)) {  // some row of the wave explores (about epsilon of the rows)
        // Per 64-task window: the row's availability in task order, assembled from its 4
        // lanes with two swaps; the exploring lane then takes the target-th set bit by a
        // popcount bisection.
        const int nwin = (nct + 3) / 4;
        int target = -1, found = -1;
        for (int ntt = 0; ntt < NT; ++ntt) {
            const bool mine_row = explore && nt == ntt;
            int cnt = __popcll(amask[ntt][0]) + (GEN ? __popcll(amask[ntt][1]) : 0);
            {
                const SwapPair c16 = swap16((uint32_t)cnt);
                const SwapPair c32 = swap32(c16.a + c16.b);
                cnt = (int)(c32.a + c32.b);
            }
            if (mine_row) {
                if (cnt == 0) atomicCAS(sel.err, 0, ASG_E_INVALID_ARG);
                else target = (int)(((uint64_t)rr.y * (uint64_t)cnt) >> 32);
            }
            for (int w = 0; w < nwin; ++w) {
                const uint32_t mine = (uint32_t)(((GEN && w >= 4) ? amask[ntt][1] : amask[ntt][0]) >> (16 * (w & 3))) & 0xFFFFu;
                uint32_t lo = 0, hi = 0;  // this lane's tasks of the window, in task order
#pragma unroll
                for (int c = 0; c < 2; ++c) lo |= ((mine >> (4 * c)) & 0xFu) << (16 * c + 4 * q);
#pragma unroll
                for (int c = 2; c < 4; ++c) hi |= ((mine >> (4 * c)) & 0xFu) << (16 * (c - 2) + 4 * q);
                const SwapPair l16 = swap16(lo), h16 = swap16(hi);
                const SwapPair l32 = swap32(l16.a | l16.b), h32 = swap32(h16.a | h16.b);
                uint64_t row_mask = (uint64_t)(l32.a | l32.b) | ((uint64_t)(h32.a | h32.b) << 32);
                if (mine_row && target >= 0) {
                    const int pc = __popcll(row_mask);
                    if (target < pc) {
                        int k = target, pos = 0;
#pragma unroll
                        for (int half = 32; half >= 1; half >>= 1) {
                            const uint64_t low = row_mask & ((1ull << half) - 1ull);
                            const int lc = __popcll(low);
                            const bool up = k >= lc;
                            k -= up ? lc : 0;
                            pos += up ? half : 0;
                            row_mask = up ? (row_mask >> half) : low;
                        }
                        found = 64 * w + pos;
                        target = -1;
                    } else {
                        target -= pc;
                    }
                }
            }
        }
        if (found >= 0) action = found;
    }
    if (q < NT && ok[nt]) sel.out[oidx[nt]] = action;
    return action;
}

}  // namespace asg
