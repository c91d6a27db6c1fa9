/*
 * asg.h -- C-ABI of the MI355X-native batched sequential-assignment environment.
 *
 * One handle = E independent MockConstellationEnv episodes resident on one GPU,
 * advanced in lockstep by HIP kernels that read actions from, and write observations,
 * rewards, masks and bookkeeping into, an EpisodeBatch whose tensors the CALLER owns
 * (PyTorch tensors; zero copies).  Every entry point is stream-ordered and asynchronous
 * to the host unless stated otherwise, returns 0 on success or a negative ASG_E_* code,
 * and never throws across the boundary; asg_last_error() explains the last failure.
 *
 * Reference interfaces replaced (all paths under /root/reference/src):
 *   asg_create / asg_destroy   MockConstellationEnv.__init__ / close
 *                              (envs/mock_constellation_env.py:17-65, :177-178), one
 *                              instance per env of ParallelRunner.__init__
 *                              (runners/parallel_runner.py:14-31)
 *   asg_reset                  MockConstellationEnv.reset + get_pretransition_data
 *                              (mock_constellation_env.py:94-114, :164-175) and the
 *                              runner's batch.update(pre_transition_data, ts=0)
 *                              (episode_runner.py:55-74, parallel_runner.py:94-111)
 *   asg_step                   MockConstellationEnv.step (mock_constellation_env.py:116-162)
 *                              + the runner's post-/pre-transition batch.update calls and
 *                              OneHot preprocess (episode_runner.py:80-95,
 *                              parallel_runner.py:141-200, components/episode_buffer.py:89-129,
 *                              components/transforms.py:12-22)
 *   asg_random_actions         a uniform random policy (BASELINE configs[1])
 *   asg_random_rollout         that policy's episode (reset + T x (actions + step)) in one launch
 *   asg_set_benefits           MockConstellationEnv(sat_prox_mat=...) injection
 *                              (mock_constellation_env.py:22, :32-37)
 *   asg_beta_hat               MockConstellationEnv.beta_hat (mock_constellation_env.py:228-274)
 *   asg_lsa_batched            scipy.optimize.linear_sum_assignment per env, as called by
 *                              mock_constellation_env.py:122, action_selectors/sap_selectors.py:32,90,
 *                              action_selectors/non_rl_selectors.py:47
 *   asg_haa_select             HAASelector.select_action (action_selectors/non_rl_selectors.py:19-50)
 *   asg_sap_select             SequentialAssignmentProblemSelector.select_action
 *                              (action_selectors/sap_selectors.py:52-98): noise + LSA per env
 *   asg_epsilon_greedy         EpsilonGreedyActionSelector.select_action
 *                              (action_selectors/classic_selectors.py:28-54)
 *   asg_rnn_agent_forward      RNNAgent.forward (modules/agents/rnn_agent.py:23-31) as called by
 *                              BasicMAC.forward for action selection (basic_controller.py:26-48)
 *   asg_get_returns            the runners' episode_return accumulation
 *                              (episode_runner.py:84, parallel_runner.py:173-176)
 *   asg_filtered_*             FilteredSAPActionSelector / FilteredEpsGrSAPTestActionSelector
 *                              (action_selectors/filtered_sap_selectors.py:7-148),
 *                              FilteredEpsilonGreedyActionSelector / FilteredSoftPoliciesSelector
 *                              (action_selectors/filtered_classic_selectors.py:6-103)
 *   asg_real_haal_select       HAALSelector.select_action (action_selectors/non_rl_selectors.py:54-118)
 *   asg_rollout                the runner loop select(0); for t: env.step(t) +
 *                              mac.select_actions(t + 1), fused for a range of steps up to a whole
 *                              episode (episode_runner.py:60-127 / parallel_runner.py:113-200);
 *                              asg_step_select = one step of it; asg_reset_rollout = env.reset()
 *                              (mock_constellation_env.py:94-114) + the whole loop in one launch
 */
#ifndef ASG_H
#define ASG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ASG_ABI_VERSION 1

/* ---- status codes ---------------------------------------------------------------- */
#define ASG_OK 0
#define ASG_E_INVALID_ARG (-1)   /* maps to ValueError in the Python shim */
#define ASG_E_HIP (-2)           /* HIP runtime failure -> RuntimeError */
#define ASG_E_STATE (-3)         /* call out of order (step before reset, step past T) */
#define ASG_E_LSA_INVALID (-4)   /* "matrix contains invalid numeric entries" */
#define ASG_E_LSA_INFEASIBLE (-5)/* "cost matrix is infeasible" */
#define ASG_E_ACTION_RANGE (-6)  /* an action outside [0, m) was stepped */

/* ---- element types of batch fields ------------------------------------------------- */
enum asg_dtype {
    ASG_F32 = 0,
    ASG_F64 = 1,
    ASG_I64 = 2,
    ASG_I32 = 3,
    ASG_BOOL = 4, /* 1 byte, torch.bool */
    ASG_F16 = 5,  /* IEEE half (RealConstellationEnv scheme) */
    ASG_I16 = 6,
};

/* A strided view of one EpisodeBatch field.  ptr addresses element [0, 0, 0, 0] of the
 * [B, T+1, d2, d3] tensor; strides are in ELEMENTS (torch .stride()), unused trailing
 * dims have size 1.  ptr == NULL means "field absent, skip the write". */
typedef struct {
    void *ptr;
    int32_t dtype;
    int32_t pad_;
    int64_t stride[4];
} asg_field;

/* The transition_data of an EpisodeBatch (components/episode_buffer.py:30-77) for the
 * envs of one handle.  Shapes per scheme (mock_constellation_env.py:73-86):
 *   obs           f32  [B, T+1, n, m*(L+1)]
 *   actions       i64  [B, T+1, n, 1]      (f32 [B, T+1, n, m] bids when bids_as_actions)
 *   avail_actions bool [B, T+1, n, m]
 *   rewards       f32  [B, T+1, n]
 *   terminated    bool [B, T+1, 1]
 *   prev_assigns  i64  [B, T+1, n]
 *   beta          f32  [B, T+1, n, m]
 *   actions_onehot i64 [B, T+1, n, m]     (OneHot keeps the input dtype, transforms.py:21-22)
 *   filled        i64  [B, T+1, 1]                                                         */
typedef struct {
    asg_field obs, actions, avail_actions, rewards, terminated, prev_assigns, beta,
        actions_onehot, filled;
} asg_batch_view;

/* ---- configuration ------------------------------------------------------------------ */
enum asg_rng_mode {
    ASG_RNG_PHILOX = 0,   /* native: counter-based Philox4x32-10 keyed (seed, global env, episode) */
    ASG_RNG_MT19937 = 1,  /* compat: numpy legacy MT19937 stream per env, bit-exact draws */
};

enum asg_benefit_mode {
    ASG_BENEFIT_BUMP = 0,     /* generate_benefits_over_time bumps (~25% active pairs) */
    ASG_BENEFIT_DENSE = 1,    /* every (i, j) pair active (BASELINE config 5) */
    ASG_BENEFIT_INJECTED = 2, /* constant table from asg_set_benefits (sat_prox_mat=) */
};

/* reference quirks (SURVEY.md §8(a) "quirks"); 0 = native semantics */
#define ASG_QUIRK_PREV_ASSIGNS_ZERO 0x1u   /* batch prev_assigns never written (mock :170-174) */
#define ASG_QUIRK_PARALLEL_TERMINATED 0x2u /* ParallelRunner terminated flag bug (parallel_runner.py:181-187) */
#define ASG_QUIRK_REPLICATE_STREAM 0x4u    /* every env shares env 0's MT stream (forked workers) */

typedef struct {
    int64_t num_envs;       /* E: envs owned by this handle (one GPU) */
    int32_t n, m, T, L;     /* agents, tasks, horizon, lookahead */
    double lambda_;         /* handover penalty */
    int32_t bids_as_actions;
    int32_t rng_mode;       /* asg_rng_mode */
    int32_t benefit_mode;   /* asg_benefit_mode */
    uint32_t quirks;        /* ASG_QUIRK_* */
    uint64_t seed;
    int64_t env_index_base; /* global index of env 0 (rank * E when sharded) */
    const double *T_trans;  /* host [m][m] transition-penalty matrix or NULL = 1 - I (mock :40) */
} asg_config;

typedef struct asg_handle asg_handle;

/* ---- lifecycle ---------------------------------------------------------------------- */
int asg_abi_version(void);
const char *asg_last_error(const asg_handle *h); /* h may be NULL: last global error */
int asg_create(const asg_config *cfg, int device, void *hip_stream, asg_handle **out);
int asg_destroy(asg_handle *h);
int asg_set_stream(asg_handle *h, void *hip_stream);

/* ---- the hot path --------------------------------------------------------------------- */
/* New episode: draw benefits (unless injected) and initial prev_assigns, zero returns,
 * write pre-transition row `ts` (obs, beta, avail_actions, prev_assigns, filled). */
int asg_reset(asg_handle *h, const asg_batch_view *b, int ts);
/* One transition of every env: read actions at row ts; write rewards/terminated/
 * actions_onehot at ts and obs/beta/avail_actions/prev_assigns/filled at ts+1;
 * accumulate per-env float64 returns.  Actions outside [0, m) set a sticky device
 * error reported by asg_sync_status. */
int asg_step(asg_handle *h, const asg_batch_view *b, int ts);
/* asg_step with flags.  ASG_STEP_USE_SELECTED_BIDS (bids_as_actions): the caller states that
 * batch row ts still holds exactly the bids asg_bids_select wrote there (nothing wrote the row
 * since), so the step takes the assignments that call solved instead of solving the row again;
 * ASG_E_STATE when row ts is not the row asg_bids_select last wrote (a step or reset came in
 * between, or another row / layout).  Without the flag (asg_step) the bids row is always
 * solved as it is at the step (mock_constellation_env.py:121-122). */
#define ASG_STEP_USE_SELECTED_BIDS 0x1
int asg_step_ex(asg_handle *h, const asg_batch_view *b, int ts, int flags);
/* Uniform random actions in [0, m) at row ts (Philox keyed (seed, env, episode, t)). */
int asg_random_actions(asg_handle *h, const asg_batch_view *b, int ts);
/* The random policy's episode in one launch: for the next `steps` steps of every env, the
 * actions asg_random_actions draws (written at rows ts ..) and the transitions asg_step makes
 * (rows ts .. ts + steps); reset != 0 first runs asg_reset's reset into row ts (not in the
 * MT19937 mode: its reset is asg_reset).  Results equal asg_reset + steps x
 * (asg_random_actions + asg_step), bit for bit (episode_runner.py:60-100 with a uniform
 * policy over mock_constellation_env.py:94-162). */
int asg_random_rollout(asg_handle *h, const asg_batch_view *b, int ts, int steps, int reset);
/* Blocks until the handle's stream drains; returns the first sticky device error. */
int asg_sync_status(asg_handle *h);

/* ---- state in / out ------------------------------------------------------------------- */
/* Constant benefit table, reference layout [E][n][m][T] float64 (host or device ptr). */
int asg_set_benefits(asg_handle *h, const double *table, int64_t count, int on_device);
/* The current episode's benefit table [E][n][m][T] float64 into a device buffer
 * (materialises Philox/bump draws in float64; a debugging and parity aid). */
int asg_export_benefits(asg_handle *h, double *out_dev);
/* Philox modes: the current episode's bump parameters [E][n][m][3] float32 (scale -- 0 for an
 * inactive pair --, center, a2) into a device buffer: value(t) = scale * 2^(-(t - center)^2 * a2),
 * a2 = log2(e) / (2 sigma_2) (mock_constellation_env.py:293).  Observations and beta hold a
 * float32 evaluation within 1e-6 relative of the float64 value (exp results below FLT_MIN
 * flush to 0); rewards,
 * the beta_hat mask and asg_export_benefits use the float64 evaluation. */
int asg_export_bump_params(asg_handle *h, float *out_dev);
/* Current internal prev_assigns [E][n] (int64, device buffer). */
int asg_export_prev_assigns(asg_handle *h, int64_t *out_dev);
/* Per-env float64 returns accumulated since the last reset [E] (device buffer). */
int asg_get_returns(asg_handle *h, double *out_dev);
/* Current step counter k of the handle (host value; 0 after reset). */
int asg_get_step(const asg_handle *h, int *k_out);
/* Advance every env's MT19937 stream by `words` 32-bit draws (compat mode): models
 * other consumers of numpy's global stream between resets (jumpstart_controller.py:33). */
int asg_advance_stream(asg_handle *h, int64_t words);

/* ---- batched kernels for the action selectors ----------------------------------------- */
/* beta_hat for a batch of states: beta [B][n][m] (f32 or f64, strides in elements),
 * prev [B][n] int64 -> out [B][n][m] float64.  T_trans: device [m][m] f64 or NULL. */
int asg_beta_hat(const void *beta, int beta_dtype, const int64_t beta_strides[3],
                 const int64_t *prev, const int64_t prev_strides[2], int64_t B, int n, int m,
                 const double *T_trans_dev, double lambda_, double *out, void *hip_stream);
/* scipy-exact linear_sum_assignment on B cost matrices C[b] = [nr][nc] (f32 or f64,
 * element strides {batch, row, col}).  row_out/col_out: [B][min(nr, nc)] int64 device
 * buffers; status_out [B] int32 device buffer (0, ASG_E_LSA_INVALID, ASG_E_LSA_INFEASIBLE).
 * Either of row_out / status_out may be NULL. */
int asg_lsa_batched(const void *C, int dtype, const int64_t strides[3], int64_t B, int nr,
                    int nc, int maximize, int64_t *row_out, int64_t *col_out,
                    int32_t *status_out, void *hip_stream);
/* HAASelector: per env LSA(maximize) of beta_hat(beta[b], prev[b]) -> col_out [B][n]
 * float32 (the selector returns float tensors holding task ids, non_rl_selectors.py:30). */
int asg_haa_select(const float *beta, const int64_t beta_strides[3], const int64_t *prev,
                   const int64_t prev_strides[2], int64_t B, int n, int m,
                   const double *T_trans_dev, double lambda_, float *col_out,
                   int32_t *status_out, void *hip_stream);

/* SequentialAssignmentProblemSelector (sap_selectors.py:52-98) for n <= m <= 64, fused:
 * per env b, std = mean(|Q[b]|) * epsilon * 2 (float32), Q' = Q[b] + N(0, std^2) noise
 * (Philox keyed by (seed, env_index_base + b, counter), Box-Muller; exactly zero noise when
 * epsilon == 0), col_out[b] = LSA(Q', maximize)[1] as float32 task ids (the selector's
 * float picked_actions).  Q [B][n][m] f32, any strides.  status_out [B] int32 (0,
 * ASG_E_LSA_INVALID for NaN / +inf entries, ASG_E_LSA_INFEASIBLE), may be NULL; failed envs
 * get -1 rows.  ASG_E_INVALID_ARG when n > m or m > 64 (the Python selector then adds the
 * noise with torch and calls asg_lsa_batched).  Square problems (n == m) are solved by a
 * certified fast path (column reduction + shortest augmenting paths, kept only when the
 * final duals prove the optimum unique by a margin far above float64 rounding, so that
 * scipy's assignment is the same one), the others and every uncertified problem by the
 * scipy-exact solver.  path_steps_out [B] int32 (may be NULL): an instrumented instance also
 * writes each env's count of augmenting-path steps, the fast path's in bits 0..15 and the
 * scipy-exact solver's (scipy's inner-loop iterations) in bits 16..30, for the LSA
 * efficiency figure; same assignments. */
int asg_sap_select(const float *q, const int64_t q_strides[3], int64_t B, int n, int m,
                   double epsilon, uint64_t seed, uint64_t counter, int64_t env_index_base,
                   float *col_out, int32_t *status_out, int32_t *path_steps_out, void *hip_stream);
/* asg_sap_select writing the assignment as the int64 actions the runner's batch.update casts
 * the selector's float picked_actions to (parallel_runner.py:150-152, episode_buffer.py:89-129):
 * act_out [B][n] int64 contiguous (e.g. a time-major EpisodeBatch actions row), -1 rows for
 * failed envs.  Same draws and assignments as asg_sap_select.  status_out [B] (may be NULL)
 * ACCUMULATES: status_out[b] = min(status_out[b], status of env b) -- zero it once, read it
 * once per episode (error codes are negative). */
int asg_sap_select_into(const float *q, const int64_t q_strides[3], int64_t B, int n, int m,
                        double epsilon, uint64_t seed, uint64_t counter, int64_t env_index_base,
                        int64_t *act_out, int32_t *status_out, int32_t *path_steps_out, void *hip_stream);
/* asg_sap_select_into with the certified fast path warm-started (square problems): duals
 * [B][64] float64 (device, 8-B aligned) holds each env's column duals from its previous call
 * and receives this call's (NaN for an env whose fast path did not finish); warm = 0 ignores
 * the input (the first call).  Same assignments as asg_sap_select_into -- scipy's, whatever
 * duals the search starts from (the result is used only under the uniqueness certificate,
 * else the scipy-exact solver runs) -- in fewer augmenting-path steps on consecutive steps'
 * SAP Q-values (sap_selectors.py:60-98 called once per step of an episode). */
int asg_sap_select_warm(const float *q, const int64_t q_strides[3], int64_t B, int n, int m,
                        double epsilon, uint64_t seed, uint64_t counter, int64_t env_index_base,
                        int64_t *act_out, int32_t *status_out, int32_t *path_steps_out, double *duals,
                        int warm, void *hip_stream);
/* The matrix asg_sap_select solves for the same arguments: q_out [B][n][m] f32 contiguous =
 * Q + the selector's noise (parity tooling: the selection at epsilon > 0 is checked against
 * scipy on it).  status_out [B] (may be NULL): 0 or ASG_E_LSA_INVALID. */
int asg_sap_noise(const float *q, const int64_t q_strides[3], int64_t B, int n, int m,
                  double epsilon, uint64_t seed, uint64_t counter, int64_t env_index_base,
                  float *q_out, int32_t *status_out, void *hip_stream);

/* epsilon-greedy over Q [B][n][m] (f32) with availability mask avail [B][n][m] (bool):
 * per row, with probability epsilon a uniformly random available action, else the first
 * maximal available Q (NaN propagates as in torch.max).  Randomness: Philox keyed by
 * (seed, counter, global row = (env_index_base + b) * n + i), so a rank holding envs
 * [env_index_base, env_index_base + B) draws exactly what a 1-GPU run draws for them.
 * out [B][n] int64 (strided, e.g. the EpisodeBatch actions row);
 * status [1] int32 device word set to ASG_E_INVALID_ARG if a row with no available action
 * had to explore (torch's Categorical would raise).  May be NULL. */
int asg_epsilon_greedy(const float *q, const int64_t q_strides[3], const uint8_t *avail,
                       const int64_t avail_strides[3], int64_t B, int n, int m, double epsilon,
                       uint64_t seed, uint64_t counter, int64_t env_index_base, int64_t *out,
                       const int64_t out_strides[2], int32_t *status, void *hip_stream);

/* RNNAgent forward (inference) for R agent rows in one fused f32-MFMA kernel:
 *   x = relu(X W1^T + b1); GRUCell(x, h) (use_rnn) or relu(x W_ih^T + b_ih); q = h' W2^T + b2.
 * Weights are first packed (asg_rnn_agent_pack, once per weight update) from the torch
 * nn.Linear / nn.GRUCell layouts (W1 [hidden][K], W_ih / W_hh [3*hidden][hidden] -- or
 * W_ih = W_rnn [hidden][hidden] and W_hh = NULL when use_rnn = 0 -- and W2 [n_out][hidden])
 * into a device buffer of asg_rnn_agent_packed_size() bytes.
 * X [R][K] f32, any K >= 1 and row stride x_stride (>= K, or 0 = one row broadcast to all;
 * float4 row loads when K, x_stride and
 * x are 16-B aligned, guarded scalar loads otherwise); h_in [R][hidden] with row stride
 * h_stride (% 4 == 0, 16-B aligned; 0 = one row broadcast to all, NULL = zeros); biases
 * contiguous.  Outputs h_out [R][hidden], q_out [R][n_out], contiguous.  hidden must be 64,
 * 1 <= n_out <= 512 (the real envs' m, e.g. 450; a partial last 16-task tile is masked). */
int64_t asg_rnn_agent_packed_size(int K, int hidden, int n_out, int use_rnn);
/* Which layers of this build run their f32 products as three-way-split bf16 MFMAs (six cross
 * products, fp32-level accuracy; asg_agent.hip): bit 0 = GRU (default), bit 1 = fc1.  The
 * rest run f32 MFMAs.  For roofline accounting (bench.py); results match either way. */
int asg_rnn_agent_mfma_mode(void);
/* The MFMA mode of the kernel asg_rnn_agent_forward / _select run for this shape (16-B
 * aligned rows): 4 = every layer's f32 products on two-way-split f16 MFMAs (the split-f16
 * kernel: GRU, K % 32 == 0, n_out % 16 == 0, 16 <= n_out <= 256; accuracy vs float64 at or
 * below PyTorch fp32's, tests/test_gpu_agent.py), else asg_rnn_agent_mfma_mode(). */
int asg_rnn_agent_mode(int K, int hidden, int n_out, int use_rnn);
int asg_rnn_agent_pack(const float *W1, const float *W_ih, const float *W_hh, const float *W2, int K,
                       int hidden, int n_out, int use_rnn, void *packed, void *hip_stream);
int asg_rnn_agent_forward(const float *x, int64_t x_stride, int64_t R, int K, const float *h_in,
                          int64_t h_stride, const void *packed, const float *b1, const float *b_ih,
                          const float *b_hh, const float *b2, int hidden, int n_out, int use_rnn,
                          float *h_out, float *q_out, void *hip_stream);
/* asg_rnn_agent_forward + asg_epsilon_greedy fused: the Q tile never leaves the chip
 * (q_out may be NULL).  Rows are (env, agent) = (row / n, row % n); avail [env][agent][m]
 * bool with strides avail_strides = {env, agent} (task stride 1); actions written to
 * out[env * out_strides[0] + agent * out_strides[1]] (int64).  Same Philox stream as
 * asg_epsilon_greedy for equal (seed, counter, env_index_base): identical actions. */
int asg_rnn_agent_select(const float *x, int64_t x_stride, int64_t R, int K, const float *h_in,
                         int64_t h_stride, const void *packed, const float *b1, const float *b_ih,
                         const float *b_hh, const float *b2, int hidden, int n_out, int use_rnn,
                         float *h_out, float *q_out, const uint8_t *avail,
                         const int64_t avail_strides[2], int n, double epsilon, uint64_t seed,
                         uint64_t counter, int64_t env_index_base, int64_t *out,
                         const int64_t out_strides[2], int32_t *status, void *hip_stream);

/* ---- filtered selectors (the real-env algorithms' action_selector) -------------------------
 * The agent emits M + 1 values per agent: its top-M tasks by total benefit and a baseline.
 * asg_filtered_topm: per (env, agent) row, total[j] = beta[b][i][j][:].sum() in beta's dtype
 * (float16: float32 accumulation left to right, rounded to half -- torch's Half sum; float32 /
 * float64 left to right), and the M largest task ids in descending order, ties to the lower
 * index (th.topk(total_beta, k=M).indices, filtered_sap_selectors.py:24,52; torch leaves tie
 * order unspecified; NaN ranks first).  beta strides {env, agent, task, l} in elements;
 * topm_out [B][n][M] int64 contiguous.  m <= 1024, 1 <= M <= min(m, 64). */
int asg_filtered_topm(const void *beta, int beta_dtype, const int64_t beta_strides[4], int64_t B, int n, int m,
                      int L, int M, int64_t *topm_out, void *hip_stream);
/* The filtered selectors' benefit matrix (filtered_sap_selectors.py:37-55,
 * filtered_classic_selectors.py:37-54): mat[b][i][j] = q[b][i][M] + float32(u * 1e-8f), then
 * mat[b][i][topm[b][i][s]] = q[b][i][s] for s < M.  u: tie_noise [B][n][m] f32 (the reference's
 * th.rand_like draws, parity mode) or NULL = Philox uniforms keyed (seed, env_index_base + b,
 * counter).  FilteredSAPActionSelector's exploration: gauss_noise [B][n][m] f32 added as given,
 * or, when NULL and gauss_epsilon > 0, N(0, std^2) per env with std = float32(mean|mat[b]| *
 * eps) * 2 (Philox Box-Muller; n <= 8188 agents: the per-agent sums stay in 64 KiB of LDS, else
 * ASG_E_INVALID_ARG -- pass gauss_noise for larger n).  q [B][n][M+1] f32 any strides; mat_out
 * [B][n][m] contiguous. */
int asg_filtered_benefits(const float *q, const int64_t q_strides[3], const int64_t *topm, int64_t B, int n, int m,
                          int M, const float *tie_noise, double gauss_epsilon, const float *gauss_noise,
                          uint64_t seed, uint64_t counter, int64_t env_index_base, float *mat_out,
                          void *hip_stream);
/* asg_epsilon_greedy over the benefit matrix with the argmax NOT masked by availability
 * (benefit_matrix.max(dim=2)[1], filtered_classic_selectors.py:57-61); exploration draws a
 * uniformly random available task (Categorical(avail)) exactly as asg_epsilon_greedy. */
int asg_filtered_epsilon_greedy(const float *mat, const int64_t mat_strides[3], const uint8_t *avail,
                                const int64_t avail_strides[3], int64_t B, int n, int m, double epsilon,
                                uint64_t seed, uint64_t counter, int64_t env_index_base, int64_t *out,
                                const int64_t out_strides[2], int32_t *status, void *hip_stream);
/* FilteredSoftPoliciesSelector's index -> task map (filtered_classic_selectors.py:79-101):
 * picked [B][n] int64 in [0, M]: p < M -> topm[b][i][p]; p == M -> a uniformly random task
 * outside the top M (Philox keyed (seed, env_index_base + b, counter, agent)).  out [B][n]
 * int64; status [1] int32 device word set to ASG_E_INVALID_ARG for a picked index outside
 * [0, M]. */
int asg_filtered_soft_map(const int64_t *picked, const int64_t *topm, int64_t B, int n, int m, int M,
                          uint64_t seed, uint64_t counter, int64_t env_index_base, int64_t *out,
                          int32_t *status, void *hip_stream);

/* Fused rollout: `steps` transitions of every env (asg_step semantics, k = the handle's
 * step .. k + steps - 1, batch rows ts ..) with the agent forward + epsilon-greedy selection
 * (asg_rnn_agent_select semantics) of the rows in between, in ONE kernel -- the runner loop
 * select(0); for t: env.step(t), mac.select_actions(t + 1) (episode_runner.py:60-127,
 * parallel_runner.py:113-200).  select_first: also select on row ts (the reset row; k == 0
 * only) before the first transition; select_last: also select on the row after the last
 * transition (needs k + steps < T).  Row k + 1 is selected when k + 1 < T and it is not the
 * last row without select_last.  A whole episode is asg_reset then
 * asg_rollout(ts = 0, steps = T, select_first = 1, select_last = 0).  The observation rows
 * are generated in the agent's operand layout, written to the batch and consumed without
 * being read back; each env's selected / previous tasks stay in the kernel's LDS between
 * steps.  Batch contents, returns, hidden state and actions equal the separate
 * asg_step / asg_rnn_agent_select calls with the same arguments (counter, counter + 1, ...
 * for the selections in row order).  Requirements: Philox bump/dense benefits, integer
 * actions, 16 <= m <= 256, n <= 256, L >= 1, the RNNAgent with hidden 64 (use_rnn: GRUCell,
 * b_r0 / b_r1 = b_ih / b_hh; else Linear + ReLU, b_r0 = its bias, b_r1 unused) on K = m (L + 1)
 * inputs, weights packed by asg_rnn_agent_pack for n_out = m, and a contiguous time-major
 * EpisodeBatch.  h_in [E n][64] (row stride h_stride, 0 = one broadcast row, NULL = zeros)
 * feeds the first selection; h_out [E n][64] receives every later one's state and finally
 * the last selection's.  hip_stream NULL = the handle's stream. */
int asg_rollout(asg_handle *h, const asg_batch_view *b, int ts, int steps, int select_first, int select_last,
                const void *packed, const float *b1, const float *b_r0, const float *b_r1, const float *b2, int K,
                int hidden, int use_rnn, const float *h_in, int64_t h_stride, float *h_out, double epsilon,
                uint64_t seed, uint64_t counter, int32_t *status, void *hip_stream);
/* asg_reset(ts) then asg_rollout(ts, steps, select_first = 1, select_last) in ONE launch: the
 * reset (a fresh Philox episode key, prev_assigns from the permutation draw, returns = 0, the
 * pre-transition row ts) runs in the rollout kernel's env prologue and its first selection
 * pass, which stores the reset row it generates.  Batch, returns, hidden state and actions
 * equal asg_reset + asg_rollout.  Philox bump/dense benefits only. */
int asg_reset_rollout(asg_handle *h, const asg_batch_view *b, int ts, int steps, int select_last, const void *packed,
                      const float *b1, const float *b_r0, const float *b_r1, const float *b2, int K, int hidden,
                      int use_rnn, const float *h_in, int64_t h_stride, float *h_out, double epsilon, uint64_t seed,
                      uint64_t counter, int32_t *status, void *hip_stream);
/* asg_rollout with steps = 1, select_first = 0, select_last = 1 and the GRU agent: asg_step
 * at row ts then asg_rnn_agent_select for row ts + 1 (the round-2 per-step entry point). */
int asg_step_select(asg_handle *h, const asg_batch_view *b, int ts, const void *packed, const float *b1,
                    const float *b_ih, const float *b_hh, const float *b2, int K, int hidden, const float *h_in,
                    int64_t h_stride, float *h_out, double epsilon, uint64_t seed, uint64_t counter,
                    int32_t *status, void *hip_stream);
/* asg_step at row ts then the agent forward (asg_rnn_agent_forward semantics) on row ts + 1,
 * in one rollout-kernel launch: the runner loop's env.step(t) + mac.forward(t + 1) for a
 * selector that acts on Q outside the kernel (SequentialAssignmentProblemSelector,
 * mock_constellation_reda.yaml; sap_selectors.py:52-98).  Observation row ts + 1 is generated,
 * stored and consumed on chip; q_out [E n][m] f32 contiguous (16-B aligned) receives the Q rows,
 * h_out the hidden state.  Needs k + 1 < T; the actions of row ts are read from the batch.
 * Every benefit source (Philox, MT19937-compat and injected tables); agent and batch
 * requirements as asg_rollout.  bids_as_actions: the tasks of row ts are LSA(bids row ts,
 * maximize), solved in the launch's stream order before the transition; asg_step_forward_ex
 * with ASG_STEP_USE_SELECTED_BIDS takes the assignments asg_bids_select solved for that row
 * instead (as asg_step_ex). */
int asg_step_forward(asg_handle *h, const asg_batch_view *b, int ts, const void *packed, const float *b1,
                     const float *b_r0, const float *b_r1, const float *b2, int K, int hidden, int use_rnn,
                     const float *h_in, int64_t h_stride, float *h_out, float *q_out, void *hip_stream);
int asg_step_forward_ex(asg_handle *h, const asg_batch_view *b, int ts, const void *packed, const float *b1,
                        const float *b_r0, const float *b_r1, const float *b2, int K, int hidden, int use_rnn,
                        const float *h_in, int64_t h_stride, float *h_out, float *q_out, int flags,
                        void *hip_stream);
/* asg_reset then the agent forward on the reset row ts (Q to q_out, the hidden state to h_out), in
 * one launch: the runner's env.reset() + mac.forward(0) of a selector acting on Q outside the
 * kernel (runners/episode_runner.py:49-62 with sap_selectors.py:52-98 / bet_selectors.py).  The
 * reset row is generated, stored and consumed on chip.  Philox bump / dense benefits and the
 * MT19937 mode (its draw kernels first, as asg_reset_rollout); not an injected table under
 * Philox (asg_reset).  Same batch, Q and hidden state as asg_reset + asg_rnn_agent_forward. */
int asg_reset_forward(asg_handle *h, const asg_batch_view *b, int ts, const void *packed, const float *b1,
                      const float *b_r0, const float *b_r1, const float *b2, int K, int hidden, int use_rnn,
                      const float *h_in, int64_t h_stride, float *h_out, float *q_out, void *hip_stream);
/* bids_as_actions with the ContinuousActionSelector (config/algs/ippo_sap.yaml), replacing the
 * per-env chain BasicMAC.forward's pi_logits softmax (controllers/basic_controller.py:37-46) ->
 * ContinuousActionSelector.select_action (action_selectors/bet_selectors.py:12-20: softmax over
 * the agents, th.normal(x, std)) -> the env step's scipy LSA of the bids
 * (envs/mock_constellation_env.py:121-122), for every env of the handle in one launch (n <= m <= 64):
 * q [E][n][m] f32 (element strides) = the agent outputs; row_softmax: softmax over the tasks first
 * (agent_output_type "pi_logits"); col_softmax: softmax over the agents (softmax_agent_inputs);
 * noise_std >= 0: Gaussian noise N(0, noise_std) from Philox keyed by (seed, global env index, counter)
 * (0: the means exactly).  Writes the bids to bids_out [E][n][m] (element strides: the batch's
 * actions row) and their LSA(maximize) assignments into the handle, which asg_step_ex /
 * asg_step_forward_ex with ASG_STEP_USE_SELECTED_BIDS on that batch row use instead of solving
 * it again (the caller vouches that nothing rewrote the row in between).  A NaN / +inf bid sets
 * the env's sticky error (asg_sync_status: "matrix contains invalid numeric entries"). */
int asg_bids_select(asg_handle *h, const float *q, const int64_t q_strides[3], float *bids_out,
                    const int64_t out_strides[3], int row_softmax, int col_softmax, double noise_std, uint64_t seed,
                    uint64_t counter, void *hip_stream);
/* asg_bids_select on the instrumented kernel instance: path_steps_out [E] int32 (device) receives
 * every env's augmenting-path steps (the certified fast path's in bits 0..15, the scipy-exact
 * solver's above, as asg_sap_select); same bids and assignments (bench.py's efficiency figure). */
int asg_bids_select_count(asg_handle *h, const float *q, const int64_t q_strides[3], float *bids_out,
                          const int64_t out_strides[3], int row_softmax, int col_softmax, double noise_std,
                          uint64_t seed, uint64_t counter, int32_t *path_steps_out, void *hip_stream);
/* Number of fc1 weight slices (32 inputs x 64 units) the rollout kernel reads through L2
 * instead of LDS for an (n, m, L) env and agent kind, or -1 when asg_rollout does not take
 * the shape (GRU: 64 x 64, L = 3: 1; 256 x 256: 19).  asg_step_select_l2_slices = the GRU
 * agent's. */
int asg_rollout_l2_slices(int n, int m, int L, int use_rnn);
int asg_step_select_l2_slices(int n, int m, int L);

/* ==== RealConstellationEnv ======================================
 * Batched form of src/envs/real_constellation_env.py with injected benefits
 * (sat_prox_mat + graphs given: the constant-benefit path, :55-61).  Replaces
 * RealConstellationEnv.reset (:100-114), .step (:135-175), ._build_obs (:177-230),
 * .get_pretransition_data (:232-245) and .beta_hat (:259-327) for E envs per handle.
 * Batch fields use the reference scheme (:80-97): obs f16 [B,T+1,n,obs_size],
 * actions i16 [B,T+1,n,1], avail bool [B,T+1,n,m], rewards f16 [B,T+1,n] (one vector
 * per env), terminated bool, prev_assigns i16 [B,T+1,n], beta f16 [B,T+1,n,m,L]
 * (the asg_field strides cover (B, T+1, n, m); L must be contiguous), actions_onehot
 * i16 [B,T+1,n,m], filled i64.  Wider float / int dtypes are accepted too.
 * np.argsort ties (unspecified order in numpy) are broken by the lower index. */
typedef struct asg_real_handle asg_real_handle;

/* env family: RealConstellationEnv (real_constellation_env.py), RealPowerConstellationEnv
 * (real_power_constellation_env.py: per-satellite power drained 0.2 per meaningful task,
 * recharged 0.1 otherwise, dead at <= 0; power in state and obs), InterferenceConstellationEnv
 * (interference_constellation_env.py: the power dynamics plus a beam-interference reward
 * over satellites sharing a frequency band, :309-353). */
enum asg_real_variant { ASG_REAL_PLAIN = 0, ASG_REAL_POWER = 1, ASG_REAL_INTERFERENCE = 2 };

typedef struct {
    int64_t num_envs;
    int32_t n, m, T, L;        /* n = num_planes * num_sats_per_plane (n <= m); L = min(L, T) */
    int32_t N, M;              /* competitors and tasks in the observation; M even, m >= 3M/2 */
    double lambda_;
    const double *T_trans;     /* host [m][m] or NULL (= 1 - I) */
    const double *task_prios;  /* host [m] or NULL (= ones) */
    int32_t variant;           /* asg_real_variant */
    int32_t bids_as_actions;   /* actions are float32 bids [B,T+1,n,m]; the step's assignments are
                                  LSA(bids, maximize) (real_constellation_env.py:110-112, :140-142;
                                  real_power :112, :142; interference :121, :159); no one-hot */
    uint64_t seed;             /* power variants: Philox key of the reset assignments ... */
    int64_t env_index_base;    /* ... per global env index (choice(m, n, replace=False)) */
    const int32_t *sat_freq_bands;   /* host [n] (interference) */
    const double *neighbor_matrix;   /* host [m][m] (interference; integer-valued) */
} asg_real_config;

/* EpisodeBatch view of the real envs: the mock-env fields plus power_states f16 [B, T+1, n]
 * (power variants; real_power_constellation_env.py:112, NULL ptr = absent) */
typedef struct {
    asg_batch_view base;
    asg_field power_states;
} asg_real_batch_view;

int asg_real_create(const asg_real_config *cfg, int device, void *hip_stream, asg_real_handle **out);
void asg_real_destroy(asg_real_handle *h);
int asg_real_set_stream(asg_real_handle *h, void *hip_stream);
/* sat_prox_mat float64 [count][n][m][T] (reference layout), count = 1 (shared by every
 * env, the reference's constant benefits) or num_envs; host or device memory. */
int asg_real_set_benefits(asg_real_handle *h, const double *table, int64_t count, int on_device);
/* power variants: the reset's np.random.choice(m, n, replace=False) as given int64
 * [count][n] (count 1 or num_envs; exact-parity mode); NULL returns to Philox draws */
int asg_real_set_initial_assignments(asg_real_handle *h, const int64_t *prev0, int64_t count, int on_device);
int asg_real_reset(asg_real_handle *h, const asg_real_batch_view *view, int ts);
int asg_real_step(asg_real_handle *h, const asg_real_batch_view *view, int ts);
int asg_real_sync_status(asg_real_handle *h);
int asg_real_get_returns(asg_real_handle *h, double *out_device); /* float64 [E] */
int asg_real_get_step(const asg_real_handle *h, int *k_out);
/* get_obs_size (real_constellation_env.py:251-253): M*L + N*M*L + (N*M//2)*L + M; the
 * power variants add N + 1 (real_power_constellation_env.py:286-290) */
int asg_real_obs_size(int N, int M, int L);
/* HAALSelector (non_rl_selectors.py:54-118) on every env of the handle (any variant) at its
 * current step k: for each time-interval sequence of the window eff = min(L, T - k)
 * (build_time_interval_sequences, utils/methods.py:309-349; S = 2^(eff-1) sequences in the
 * reference's order, eff <= 6) the env is forked, and per interval LSA(maximize) of
 * beta_hat summed over L (float64, numpy's order) is stepped interval-length times; a
 * sequence's value is the sum of the steps' sum(rewards).  Power / interference variants: the
 * fork carries the power states (drained / recharged by its own steps,
 * real_power_constellation_env.py:170-178), beta_hat rows below 1e-12 power are zero (:343-347)
 * and each step pays the variant's reward (interference_constellation_env.py:309-353).  The action is the first
 * interval's assignment of the first best sequence (col_out [E][n] float32 task ids, the
 * selector's float picked_actions).  values_out [E][S] float64, best_out [E] int32 (index of
 * the winning sequence) and status_out [E] int32 (0 or the scipy error code of any LSA of
 * that env) may be NULL.  Stream-ordered; a device workspace is kept in the handle. */
int asg_real_haal_select(asg_real_handle *h, float *col_out, double *values_out, int32_t *best_out,
                         int32_t *status_out);
/* S = 2^(eff-1) at the handle's current step (0 once the episode is done) */
int asg_real_haal_num_sequences(const asg_real_handle *h);

#ifdef __cplusplus
}
#endif
#endif /* ASG_H */
