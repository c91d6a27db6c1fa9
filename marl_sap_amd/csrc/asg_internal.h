// asg_internal.h -- device-resident state of one handle, shared by the kernels and the
// C-ABI layer (passed to kernels by value: a few scalars plus device pointers).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/asg.h"

namespace asg {

// the thread-local message returned by asg_last_error(NULL) (asg_abi.hip)
void set_last_error(const std::string &msg);

struct EnvState {
    int64_t E;             // envs in this handle
    int n, m, T, L;
    double lambda_;
    int bids;              // bids_as_actions
    int rng_mode;          // asg_rng_mode
    int benefit_mode;      // asg_benefit_mode
    uint32_t quirks;       // ASG_QUIRK_*
    uint64_t seed;
    int64_t env_base;      // global index of env 0
    uint32_t episode;      // Philox counter: episodes reset so far (this handle)
    double wmin_init, wmax_init;  // throwaway __init__ draw widths (mock :34)
    double wmin, wmax;            // reset draw widths (mock :100)
    const double *T_trans; // device [m][m] or nullptr (= 1 - I)
    int *prev;             // [E][n] previous assignment (state for beta_hat)
    double *returns;       // [E] float64 episode returns
    double *table;         // [E][T][n][m] float64 (injected mode only)
    float *table32;        // [E][T][n][m] the benefits rounded to float32 (the rows' dtype; MT19937 / injected);
                           // MT19937 draws: COMPACT -- per (env, t) slice only the env's bump pairs, in
                           // (agent, task) order (the other pairs are exactly 0), see tmask / toff
    uint64_t *tmask;       // [E][n][W] (W = ceil(m / 64)) bump pairs of the compact table (MT19937 draws)
    int *toff;             // [E][n][W] compact index of each mask word's first pair
    uint32_t *mt;          // [E][625] MT19937 key + pos (compat mode)
    double2 *mtpar;        // [E][m][n] the reset's bump draws (center, +-spread; 0: no bump) (compat mode):
                           // the float64 benefits are mt_par_value() of these, no float64 table is kept
    int *assign;           // [E][n] LSA assignments of the bids (bids_as_actions)
    int *err;              // sticky device error code
};

// fused epsilon-greedy selection on the Q tile (EpsilonGreedyActionSelector, see
// asg_select.hip for the standalone form): rows are (env b, agent i) = (row / n, row % n)
struct SelectArgs {
    const uint8_t *avail;  // avail_actions, task stride 1
    int64_t a0, a1;        // (env, agent) strides of avail
    int n;                 // agents per env
    float epsilon;
    uint32_t k0, k1, counter;
    int64_t row_base;      // global row of row 0 (env_index_base * n): Philox keys by global row
    int64_t *out;          // actions (int64), (env, agent) strides o0, o1
    int64_t o0, o1;
    int *err;              // sticky: exploration over a row with no available action
};

hipError_t launch_reset(const asg_batch_view &bv, const EnvState &st, int ts, bool construct, hipStream_t s);
hipError_t launch_reset_draws(const EnvState &st, bool construct, hipStream_t s);
// bids_as_actions: assign_ready = st.assign already holds LSA(bids row ts) (asg_bids_select)
hipError_t launch_step(const asg_batch_view &bv, const EnvState &st, int ts, int k, hipStream_t s,
                       bool assign_ready = false);
// bids_as_actions: st.assign = LSA(bids row ts, maximize) per env
hipError_t launch_bids_assign(const asg_batch_view &bv, const EnvState &st, int ts, hipStream_t s);
hipError_t launch_random_actions(const asg_batch_view &bv, const EnvState &st, int ts, int k, hipStream_t s);
hipError_t launch_random_rollout(const asg_batch_view &bv, const EnvState &st, int ts, int k0, int steps, bool reset,
                                 hipStream_t s);
hipError_t launch_export_table(const EnvState &st, double *out, hipStream_t s);
hipError_t launch_export_bump_params(const EnvState &st, float *out, hipStream_t s);
hipError_t launch_import_table(const double *in, int64_t src_envs, const EnvState &st, hipStream_t s);
hipError_t launch_export_prev(const EnvState &st, int64_t *out, hipStream_t s);
hipError_t launch_mt_seed(const EnvState &st, hipStream_t s);
hipError_t launch_mt_advance(const EnvState &st, int64_t words, hipStream_t s);

hipError_t launch_lsa_batched(const void *C, int dtype, const int64_t strides[3], int64_t B, int nr, int nc,
                              int maximize, int64_t *row_out, int64_t *col_out, int32_t *status_out,
                              hipStream_t s);
hipError_t launch_beta_hat(const void *beta, int dtype, const int64_t bs[3], const int64_t *prev,
                           const int64_t ps[2], int64_t B, int n, int m, const double *T_trans, double lambda_,
                           double *out, hipStream_t s);
hipError_t launch_sap_select(const float *q, const int64_t qs[3], int64_t B, int n, int m, float epsilon,
                             uint64_t seed, uint32_t counter, int64_t env_base, float *col_out, int32_t *status_out,
                             int32_t *steps_out, hipStream_t s, int64_t *act_out = nullptr,
                             double *duals = nullptr, int warm = 0);
hipError_t launch_sap_noise(const float *q, const int64_t qs[3], int64_t B, int n, int m, float epsilon, uint64_t seed,
                            uint32_t counter, int64_t env_base, float *q_out, int32_t *status_out, hipStream_t s);
hipError_t launch_bids_select(const float *q, const int64_t qs[3], int64_t B, int n, int m, int row_sm, int col_sm,
                              float stdv, uint64_t seed, uint32_t counter, int64_t env_base, float *bids,
                              const int64_t os[3], int *assign, int *env_err, hipStream_t s, int32_t *steps_out = nullptr);
hipError_t launch_haa_select(const float *beta, const int64_t bs[3], const int64_t *prev, const int64_t ps[2],
                             int64_t B, int n, int m, const double *T_trans, double lambda_, float *col_out,
                             int32_t *status_out, hipStream_t s);

hipError_t launch_eps_greedy(const float *q, const int64_t qs[3], const uint8_t *avail, const int64_t as[3],
                             int64_t B, int n, int m, float epsilon, uint64_t seed, uint32_t counter,
                             int64_t row_base, int64_t *out, const int64_t os[2], int *err, hipStream_t s,
                             bool mask = true);

// filtered selectors (asg_filtered.hip)
hipError_t launch_filtered_topm(const void *beta, int dtype, const int64_t bs[4], int64_t B, int n, int m, int L, int M,
                                int64_t *topm, hipStream_t s);
hipError_t launch_filtered_matrix(const float *q, const int64_t qs[3], const int64_t *topm, int64_t B, int n, int m,
                                  int M, const float *tie, uint64_t seed, uint32_t counter, int64_t env_base,
                                  float *mat, double *rowabs, hipStream_t s);
hipError_t launch_filtered_gauss(float *mat, int64_t B, int n, int m, float epsilon, const float *gauss,
                                 uint64_t seed, uint32_t counter, int64_t env_base, hipStream_t s);
hipError_t launch_filtered_soft_map(const int64_t *picked, const int64_t *topm, int64_t B, int n, int m, int M,
                                    uint64_t seed, uint32_t counter, int64_t env_base, int64_t *out, int *err,
                                    hipStream_t s);

int64_t rnn_agent_packed_f4(int K, int nout, int use_rnn);
int stream_cus(hipStream_t s);        // CUs the stream may run on (persistent grids)
bool onehot_prefix_enabled();         // -DASG_AGENT_ONEHOT (build time, default on)
hipError_t launch_w1t_pack(const float *W1, int K, int P, float *out, hipStream_t s);

// split-f16 agent path (asg_h2.hip): input geometry -- NB blocks of P inputs, each padded to
// Pp = roundup(P, 32) (Kp = Pp NB); prefix: block 0 may be the one-hot prefix (P = n_out)
struct H2Geom {
    int K, P, NB, Pp, Kp, prefix, nout, nct;
};
H2Geom h2_geom(int K, int nout);
bool h2_ok(int K, int nout);
int64_t h2_packed_f4(int K, int nout, int use_rnn);
hipError_t launch_h2_pack(const float *W1, const float *Wih, const float *Whh, const float *W2, int K, int nout,
                          int use_rnn, float4 *packed, hipStream_t s);
hipError_t launch_h2_agent(const float *X, int64_t xs, int64_t R, int K, const float *Hin, int64_t hs,
                           const float4 *packed, const float *b1, const float *bih, const float *bhh, const float *b2,
                           int nout, int use_rnn, float *Hout, float *Q, const SelectArgs *sel, hipStream_t s);

// fused rollout (asg_h2.hip): the time-major batch fields it touches, as row-0 pointers and
// row strides in elements ([T+1][E][..] storage: row t is a contiguous [E][..] slab)
struct RolloutSlabs {
    float *obs;
    int64_t obs_row;
    float *beta;
    int64_t beta_row;
    uint8_t *avail;
    int64_t avail_row;
    int64_t *onehot;
    int64_t onehot_row;
    int64_t *act;
    int64_t act_row;
    float *rew;
    int64_t rew_row;
    int64_t *prevb;
    int64_t prevb_row;
    uint8_t *term;
    int64_t term_row;
    int64_t *filled;
    int64_t filled_row;
};
bool rollout_shape_ok(int n, int m, int L, int K);
int rollout_l2_slices(int n, int m, int L, int use_rnn);
hipError_t launch_rollout(const RolloutSlabs &sl, const EnvState &st, int ts, int k0, int steps, int select_first,
                          int select_last, int reset, const float4 *packed, const float *b1, const float *bi, const float *bh,
                          const float *b2, int use_rnn, const float *Hin, int64_t hs, float *Hout, float *Q,
                          float epsilon, uint64_t seed, uint32_t counter, int64_t row_base, int *err, hipStream_t s);
hipError_t launch_rnn_agent_pack(const float *W1, const float *Wih, const float *Whh, const float *W2, int K, int nout,
                                 int use_rnn, float4 *packed, hipStream_t s);
hipError_t launch_rnn_agent_fwd(const float *X, int64_t xs, int64_t R, int K, const float *Hin, int64_t hs,
                                const float4 *packed, const float *b1, const float *bih, const float *bhh,
                                const float *b2, int nout, int use_rnn, float *Hout, float *Q,
                                const SelectArgs *sel, hipStream_t s);
hipError_t launch_rnn_agent_select(const float *X, int64_t xs, int64_t R, int K, const float *Hin, int64_t hs,
                                   const float4 *packed, const float *b1, const float *bih, const float *bhh,
                                   const float *b2, int nout, int use_rnn, float *Hout, float *Q,
                                   const uint8_t *avail, int64_t a0, int64_t a1, int n, float epsilon, uint64_t seed,
                                   uint32_t counter, int64_t row_base, int64_t *out, int64_t o0, int64_t o1, int *err,
                                   hipStream_t s);

}  // namespace asg
