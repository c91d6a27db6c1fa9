// asg_agent.hip -- fused RNNAgent forward for action selection (gfx950, f32 MFMA).
//
// RNNAgent.forward (modules/agents/rnn_agent.py:23-31) over all B*n agent rows of one
// env step, in ONE pass over the observation slab:
//     x  = relu(obs @ W1^T + b1)
//     gi = x @ W_ih^T + b_ih ; gh = h @ W_hh^T + b_hh            (use_rnn: GRUCell)
//     r = sigmoid(gi_r + gh_r); z = sigmoid(gi_z + gh_z); n = tanh(gi_n + r * gh_n)
//     h' = n + z * (h - n)
//   or h' = relu(x @ W_rnn^T + b_rnn)                             (use_rnn = False)
//     q  = h' @ W2^T + b2
// The PyTorch path runs this as 4 hipBLASLt GEMMs plus the GRU cell's elementwise kernel
// (which also writes a 5*hidden backward workspace per row): ~6 GB of HBM traffic per
// step at 64 agents x 16,384 envs.  Here every intermediate stays in registers / LDS:
// HBM sees the observation rows once, h in, h' and q out.
//
// Arithmetic: v_mfma_f32_16x16x4_f32 -- exact fp32 products, fp32 accumulation (a k-ordered
// fmaf chain), i.e. fp32 like the reference; only the summation order differs from
// hipBLASLt's.  One wave owns 32 rows (2 row tiles of 16); the K dimension is walked in
// chunks of 16 so each lane loads 4 consecutive k values as one float4 (the MFMA k slots
// of step e map to k = 16t + 4q + e, identically for A and B).
#include "asg_device.h"
#include "asg_internal.h"

namespace asg {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kRowsPerWave = 32;
constexpr int kHid = 64;          // hidden_dim
constexpr int kLdsStride = kHid + 4;  // padded row (floats) of the LDS row tiles

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float4 ldg4(const float *p, bool ok) {
    return ok ? *reinterpret_cast<const float4 *>(p) : make_float4(0.f, 0.f, 0.f, 0.f);
}
__device__ __forceinline__ float comp(const float4 &v, int e) {
    return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// Packed weight layout ("fragment order"): for W [C][K] row-major (torch nn.Linear), block
// (t, ct) holds, for lane l, W[16 ct + (l & 15)][16 t + 4 (l >> 4) .. + 3] as one float4,
// so one wave loads a whole MFMA B-operand chunk as 1 KiB of contiguous memory.  K is
// zero-padded to a multiple of 16.  Offsets (in float4) of the four matrices:
//   W1: [K16/16][4][64]; W_ih: [4][12][64]; W_hh: [4][12][64] (GRU) ; W2: [4][nq][64]
__device__ __forceinline__ int64_t pk(int t, int ct, int nct, int lane) { return ((int64_t)t * nct + ct) * 64 + lane; }

__global__ void pack_weights_kernel(const float *W, int C, int K, float4 *out) {
    const int nct = C / 16, nt = (K + 15) / 16;
    const int64_t total = (int64_t)nt * nct * 64;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int lane = (int)(i & 63);
        const int ct = (int)((i >> 6) % nct);
        const int t = (int)((i >> 6) / nct);
        const int row = 16 * ct + (lane & 15), k = 16 * t + 4 * (lane >> 4);
        float4 v;
        v.x = k + 0 < K ? W[(int64_t)row * K + k + 0] : 0.f;
        v.y = k + 1 < K ? W[(int64_t)row * K + k + 1] : 0.f;
        v.z = k + 2 < K ? W[(int64_t)row * K + k + 2] : 0.f;
        v.w = k + 3 < K ? W[(int64_t)row * K + k + 3] : 0.f;
        out[i] = v;
    }
}

// acc[rt][ct] += A(rows of `a_src`, k) * W^T(k, cols 16*ct0 .. 16*(ct0+NCT)-1) over K,
// A rows come from a row-major [32][lda] LDS tile; W is row-major [cols][K] in global.
template <int NCT>
__device__ __forceinline__ void gemm_lds_a(f32x4 (&acc)[2][NCT], const float *a_lds, int lda, const float4 *Wp,
                                           int wnct, int ct0, int K) {
    const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
    for (int t = 0; t < K / 16; ++t) {
        float4 a4[2], b4[NCT];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
            a4[rt] = *reinterpret_cast<const float4 *>(a_lds + (16 * rt + r) * lda + 16 * t + 4 * q);
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) b4[ct] = Wp[pk(t, ct0 + ct, wnct, lane)];
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct) acc[rt][ct] = mfma4(comp(a4[rt], e), comp(b4[ct], e), acc[rt][ct]);
    }
}

constexpr int kStageStride = 16 + 4;  // padded row (floats) of the per-block h' stage
constexpr int kWaveLds = 2 * kRowsPerWave * kLdsStride + kRowsPerWave * kStageStride;  // floats

// NQ = n_out / 16 output tiles of fc2 (n_out <= 64); fc2 is accumulated block by block as
// each 16-unit block of h' is produced, so h' never needs a full LDS tile.
template <bool RNN, int NQ, bool SEL>
__global__ void __launch_bounds__(256) rnn_agent_fwd_kernel(
    const float *__restrict__ X, int64_t xs, int64_t R, int K, const float *__restrict__ Hin, int64_t hs,
    const float4 *__restrict__ W1p, const float *__restrict__ b1, const float4 *__restrict__ Wihp,
    const float *__restrict__ bih, const float4 *__restrict__ Whhp, const float *__restrict__ bhh,
    const float4 *__restrict__ W2p, const float *__restrict__ b2, float *__restrict__ Hout, float *__restrict__ Q,
    SelectArgs sel) {
    extern __shared__ float s_agent[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
    float *sx = s_agent + wave * kWaveLds;                 // x = relu(fc1), [32][kLdsStride]
    float *sh = sx + kRowsPerWave * kLdsStride;            // h_in, [32][kLdsStride]
    float *sp = sh + kRowsPerWave * kLdsStride;            // h' block stage, [32][kStageStride]
    const int64_t row0 = ((int64_t)blockIdx.x * 4 + wave) * kRowsPerWave;
    if (row0 >= R) return;  // whole wave idle (no block-level barrier below)
    constexpr int nout = 16 * NQ;

    // ---- h_in -> LDS (row-major, padded) -------------------------------------------
    for (int idx = lane; idx < kRowsPerWave * kHid / 4; idx += 64) {
        const int rr = idx / (kHid / 4), c4 = (idx % (kHid / 4)) * 4;
        const int64_t row = row0 + rr;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (RNN && Hin && row < R) v = *reinterpret_cast<const float4 *>(Hin + row * hs + c4);
        *reinterpret_cast<float4 *>(sh + rr * kLdsStride + c4) = v;
    }

    // ---- selection mask, loaded early (its latency hides under fc1): bit (rt, v, c) =
    //      avail[row 16 rt + 4 q + v][task 16 c + r]
    uint32_t avbits = 0;
    // (env, agent) of row row0 + d without a 64-bit division per row
    int64_t sel_b0 = 0;
    int sel_i0 = 0;
    if (SEL) {
        sel_b0 = row0 / sel.n;
        sel_i0 = (int)(row0 - sel_b0 * sel.n);
    }
    auto env_agent = [&](int d, int64_t &b, int &i) {
        b = sel_b0;
        i = sel_i0 + d;
        while (i >= sel.n) {
            i -= sel.n;
            ++b;
        }
    };
    if (SEL) {
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int64_t row = row0 + 16 * rt + 4 * q + v;
                if (row < R) {
                    int64_t b;
                    int i;
                    env_agent(16 * rt + 4 * q + v, b, i);
                    const uint8_t *ar = sel.avail + b * sel.a0 + (int64_t)i * sel.a1;
#pragma unroll
                    for (int c = 0; c < NQ; ++c)
                        if (ar[16 * c + r]) avbits |= 1u << ((rt * 4 + v) * 4 + c);
                }
            }
    }

    // ---- fc1: x = relu(X W1^T + b1), X rows streamed from HBM ------------------------
    {
        f32x4 acc[2][4];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int ct = 0; ct < 4; ++ct) acc[rt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int64_t ra = row0 + r, rb = row0 + 16 + r;
        const bool oka = ra < R, okb = rb < R;
        const float *xa = X + (oka ? ra : 0) * xs, *xb = X + (okb ? rb : 0) * xs;
        const int nt = (K + 15) / 16;
        // two chunks in flight: chunk t is consumed while t+1 and t+2 are loading
        float4 a0[2], b0[4], a1[2], b1r[4];
        auto load = [&](int t, float4 (&a4)[2], float4 (&b4)[4]) {
            const int k = 16 * t + 4 * q;
            const bool okk = t < nt && k < K;  // K % 4 == 0 (checked on the host)
            a4[0] = ldg4(xa + k, oka && okk);
            a4[1] = ldg4(xb + k, okb && okk);
#pragma unroll
            for (int ct = 0; ct < 4; ++ct) b4[ct] = t < nt ? W1p[pk(t, ct, 4, lane)] : make_float4(0.f, 0.f, 0.f, 0.f);
        };
        load(0, a0, b0);
        load(1, a1, b1r);
        for (int t = 0; t < nt; ++t) {
            float4 a4[2] = {a0[0], a0[1]};
            float4 b4[4] = {b0[0], b0[1], b0[2], b0[3]};
#pragma unroll
            for (int i = 0; i < 2; ++i) a0[i] = a1[i];
#pragma unroll
            for (int i = 0; i < 4; ++i) b0[i] = b1r[i];
            if (t + 2 < nt) load(t + 2, a1, b1r);
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                    for (int ct = 0; ct < 4; ++ct)
                        acc[rt][ct] = mfma4(comp(a4[rt], e), comp(b4[ct], e), acc[rt][ct]);
        }
        // epilogue: C layout (col = lane & 15, row = 4 * (lane >> 4) + v)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int ct = 0; ct < 4; ++ct) {
                const int col = 16 * ct + r;
                const float bb = b1[col];
#pragma unroll
                for (int v = 0; v < 4; ++v)
                    sx[(16 * rt + 4 * q + v) * kLdsStride + col] = fmaxf(acc[rt][ct][v] + bb, 0.f);
            }
    }
    wave_sync();

    // ---- recurrent layer, one 16-unit block of h' at a time; fc2 accumulated per block -------
    f32x4 aq[2][NQ];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int c = 0; c < NQ; ++c) aq[rt][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int hb = 0; hb < 4; ++hb) {
        const int u = 16 * hb + r;
        f32x4 hp[2];
        if (RNN) {
            f32x4 gi[2][3], gh[2][3];
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int g = 0; g < 3; ++g) gi[rt][g] = gh[rt][g] = f32x4{0.f, 0.f, 0.f, 0.f};
            float4 bi[3], bh[3];
            auto wload = [&](int t, float4 (&wi)[3], float4 (&wh)[3]) {
#pragma unroll
                for (int g = 0; g < 3; ++g) {
                    wi[g] = Wihp[pk(t, 4 * g + hb, 12, lane)];
                    wh[g] = Whhp[pk(t, 4 * g + hb, 12, lane)];
                }
            };
            wload(0, bi, bh);
            for (int t = 0; t < kHid / 16; ++t) {
                float4 ax[2], ah[2], ci[3], ch[3];
#pragma unroll
                for (int g = 0; g < 3; ++g) {
                    ci[g] = bi[g];
                    ch[g] = bh[g];
                }
                if (t + 1 < kHid / 16) wload(t + 1, bi, bh);  // weights of the next chunk in flight
#pragma unroll
                for (int rt = 0; rt < 2; ++rt) {
                    ax[rt] = *reinterpret_cast<const float4 *>(sx + (16 * rt + r) * kLdsStride + 16 * t + 4 * q);
                    ah[rt] = *reinterpret_cast<const float4 *>(sh + (16 * rt + r) * kLdsStride + 16 * t + 4 * q);
                }
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                        for (int g = 0; g < 3; ++g) {
                            gi[rt][g] = mfma4(comp(ax[rt], e), comp(ci[g], e), gi[rt][g]);
                            gh[rt][g] = mfma4(comp(ah[rt], e), comp(ch[g], e), gh[rt][g]);
                        }
            }
            const float bir = bih[u], biz = bih[kHid + u], bin = bih[2 * kHid + u];
            const float bhr = bhh[u], bhz = bhh[kHid + u], bhn = bhh[2 * kHid + u];
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const float h = sh[(16 * rt + 4 * q + v) * kLdsStride + u];
                    const float rg = sigmoidf_((gi[rt][0][v] + bir) + (gh[rt][0][v] + bhr));
                    const float zg = sigmoidf_((gi[rt][1][v] + biz) + (gh[rt][1][v] + bhz));
                    const float ng = tanhf((gi[rt][2][v] + bin) + rg * (gh[rt][2][v] + bhn));
                    hp[rt][v] = ng + zg * (h - ng);
                }
        } else {
            f32x4 a2[2][1];
            a2[0][0] = a2[1][0] = f32x4{0.f, 0.f, 0.f, 0.f};
            gemm_lds_a<1>(a2, sx, kLdsStride, Wihp, 4, hb, kHid);
            const float bb = bih[u];
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int v = 0; v < 4; ++v) hp[rt][v] = fmaxf(a2[rt][0][v] + bb, 0.f);
        }
        // h' block: to HBM (hidden-state output) and to the LDS stage as fc2's A operand
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int rr = 16 * rt + 4 * q + v;
                sp[rr * kStageStride + r] = hp[rt][v];
                if (row0 + rr < R) Hout[(row0 + rr) * kHid + u] = hp[rt][v];
            }
        wave_sync();
        // q += h'[:, block] W2[:, block]^T   (K = 16: one chunk)
        {
            float4 a4[2], b4[NQ];
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
                a4[rt] = *reinterpret_cast<const float4 *>(sp + (16 * rt + r) * kStageStride + 4 * q);
#pragma unroll
            for (int c = 0; c < NQ; ++c) b4[c] = W2p[pk(hb, c, NQ, lane)];
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                    for (int c = 0; c < NQ; ++c) aq[rt][c] = mfma4(comp(a4[rt], e), comp(b4[c], e), aq[rt][c]);
        }
        wave_sync();  // the stage is rewritten by the next block
    }
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int c = 0; c < NQ; ++c) {
            const float bb = b2[16 * c + r];
#pragma unroll
            for (int v = 0; v < 4; ++v) aq[rt][c][v] += bb;
        }
    if (Q) {
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int c = 0; c < NQ; ++c)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int64_t row = row0 + 16 * rt + 4 * q + v;
                    if (row < R) Q[row * nout + 16 * c + r] = aq[rt][c][v];
                }
    }
    if (SEL) {
        // the 16 lanes of a DPP row (same q) hold the nout Q-values of one agent row
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int64_t row = row0 + 16 * rt + 4 * q + v;
                const bool live = row < R;
                int64_t b;
                int i;
                env_agent(16 * rt + 4 * q + v, b, i);
                float best = -__builtin_inff();
                int bj = 0x7fffffff;
                uint32_t rowmask[NQ];  // availability bits of this row, task 16c + lane-in-row
#pragma unroll
                for (int c = 0; c < NQ; ++c) {
                    const int col = 16 * c + r;
                    const bool av = live && ((avbits >> ((rt * 4 + v) * 4 + c)) & 1u);
                    rowmask[c] = (uint32_t)(__ballot(av) >> (16 * q)) & 0xFFFFu;
                    const float x = av ? aq[rt][c][v] : -__builtin_inff();
                    if (better(x, col, best, bj)) {
                        best = x;
                        bj = col;
                    }
                }
                auto red = [&](auto perm) {
                    const float ob = __builtin_bit_cast(float, perm(__builtin_bit_cast(uint32_t, best)));
                    const int oj = (int)perm((uint32_t)bj);
                    if (better(ob, oj, best, bj)) {
                        best = ob;
                        bj = oj;
                    }
                };
                red([](uint32_t x) { return dpp32<0xB1>(x); });
                red([](uint32_t x) { return dpp32<0x4E>(x); });
                red([](uint32_t x) { return dpp32<0x141>(x); });
                red([](uint32_t x) { return dpp32<0x140>(x); });
                int action = bj == 0x7fffffff ? 0 : bj;
                if (r == 0 && live) {
                    if (sel.epsilon > 0.0f) {
                        const u32x4 rr = philox4x32_10(u32x4{(uint32_t)row, (uint32_t)(row >> 32), kCtrSelect,
                                                             sel.counter}, sel.k0, sel.k1);
                        constexpr float k2m24 = 5.9604644775390625e-08f;
                        if ((float)(rr.x >> 8) * k2m24 < sel.epsilon) {  // explore: Categorical(avail)
                            // tasks in index order j = 16 c + bit, from the row's ballot masks
                            int cnt = 0;
#pragma unroll
                            for (int c = 0; c < NQ; ++c) cnt += __popc(rowmask[c]);
                            if (cnt == 0) {
                                atomicCAS(sel.err, 0, ASG_E_INVALID_ARG);
                            } else {
                                int target = (int)(((uint64_t)rr.y * (uint64_t)cnt) >> 32);
#pragma unroll
                                for (int c = 0; c < NQ; ++c) {
                                    const int pc = __popc(rowmask[c]);
                                    if (target >= 0 && target < pc) {
                                        uint32_t msk = rowmask[c];
                                        for (int k = 0; k < target; ++k) msk &= msk - 1;  // drop lowest bits
                                        action = 16 * c + __builtin_ctz(msk);
                                    }
                                    target -= pc;
                                }
                            }
                        }
                    }
                    sel.out[b * sel.o0 + (int64_t)i * sel.o1] = action;
                }
            }
    }
}

// float4 count of the packed weight buffer
int64_t rnn_agent_packed_f4(int K, int nout, int use_rnn) {
    const int64_t w1 = (int64_t)((K + 15) / 16) * 4 * 64;
    const int64_t wr = use_rnn ? 2 * 4 * 12 * 64 : 4 * 4 * 64;
    const int64_t w2 = 4 * (int64_t)(nout / 16) * 64;
    return w1 + wr + w2;
}

hipError_t launch_rnn_agent_pack(const float *W1, const float *Wih, const float *Whh, const float *W2, int K, int nout,
                                 int use_rnn, float4 *packed, hipStream_t s) {
    float4 *p = packed;
    auto one = [&](const float *W, int C, int KK) {
        const int64_t n = (int64_t)((KK + 15) / 16) * (C / 16) * 64;
        hipLaunchKernelGGL(pack_weights_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, W, C, KK, p);
        p += n;
    };
    one(W1, kHid, K);
    if (use_rnn) {
        one(Wih, 3 * kHid, kHid);
        one(Whh, 3 * kHid, kHid);
    } else {
        one(Wih, kHid, kHid);
    }
    one(W2, nout, kHid);
    return hipGetLastError();
}

hipError_t launch_rnn_agent_fwd(const float *X, int64_t xs, int64_t R, int K, const float *Hin, int64_t hs,
                                const float4 *packed, const float *b1, const float *bih, const float *bhh,
                                const float *b2, int nout, int use_rnn, float *Hout, float *Q, const SelectArgs *sel,
                                hipStream_t s) {
    const int64_t rows_per_block = 4 * kRowsPerWave;
    const int64_t blocks = (R + rows_per_block - 1) / rows_per_block;
    const size_t lds = sizeof(float) * 4 * kWaveLds;
    const float4 *W1p = packed;
    const float4 *Wihp = W1p + (int64_t)((K + 15) / 16) * 4 * 64;
    const float4 *Whhp = Wihp + (use_rnn ? 4 * 12 * 64 : 4 * 4 * 64);
    const float4 *W2p = use_rnn ? Whhp + 4 * 12 * 64 : Whhp;
    const SelectArgs sa = sel ? *sel : SelectArgs{};
#define L_(RNN, NQ, SEL)                                                                                      \
    hipLaunchKernelGGL((rnn_agent_fwd_kernel<RNN, NQ, SEL>), dim3(blocks), dim3(256), lds, s, X, xs, R, K, Hin, hs, \
                       W1p, b1, Wihp, bih, Whhp, bhh, W2p, b2, Hout, Q, sa)
#define NQ_(RNN, SEL)                   \
    if (nq == 1) L_(RNN, 1, SEL);       \
    else if (nq == 2) L_(RNN, 2, SEL);  \
    else if (nq == 3) L_(RNN, 3, SEL);  \
    else L_(RNN, 4, SEL);
    const int nq = nout / 16;
    if (use_rnn) {
        if (sel) { NQ_(true, true) } else { NQ_(true, false) }
    } else {
        if (sel) { NQ_(false, true) } else { NQ_(false, false) }
    }
#undef NQ_
#undef L_
    return hipGetLastError();
}

hipError_t launch_rnn_agent_select(const float *X, int64_t xs, int64_t R, int K, const float *Hin, int64_t hs,
                                   const float4 *packed, const float *b1, const float *bih, const float *bhh,
                                   const float *b2, int nout, int use_rnn, float *Hout, float *Q,
                                   const uint8_t *avail, int64_t a0, int64_t a1, int n, float epsilon, uint64_t seed,
                                   uint32_t counter, int64_t *out, int64_t o0, int64_t o1, int *err, hipStream_t s) {
    const SelectArgs sa{avail, a0, a1, n, epsilon, (uint32_t)seed, (uint32_t)(seed >> 32) ^ 0x5bd1e995u, counter,
                        out, o0, o1, err};
    return launch_rnn_agent_fwd(X, xs, R, K, Hin, hs, packed, b1, bih, bhh, b2, nout, use_rnn, Hout, Q, &sa, s);
}

}  // namespace asg
