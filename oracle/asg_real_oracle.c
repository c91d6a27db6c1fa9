/* CPU restatement of the reference's RealConstellationEnv (constant-benefit path:
 * injected sat_prox_mat), reference: src/envs/real_constellation_env.py.
 *
 * TEST INFRASTRUCTURE ONLY (oracle): linked by tests/ and bench.py's CPU baseline, never
 * by the product library.  float64 throughout, the same operation order as numpy:
 *   - beta = sat_prox_mat[:, :, k:k+L] * task_prios, zero slices past T   (:110, :164-168)
 *   - total_beta = beta.sum(-1): numpy's reduce adds the L values left to right for L < 8
 *   - beta_hat: beta[..., 0] - lambda * T_trans[prev_i, j] * (beta.sum(-1) > 1e-12) (:259-327)
 *   - rewards: beta_hat[i, a_i, 0] / count(a_i) if > 0 else beta_hat[i, a_i, 0]   (:144-158)
 *   - observation builder (:177-230) with np.argsort replaced by a STABLE order: among
 *     equal keys the lower index sorts first (numpy's default quicksort leaves tie order
 *     unspecified; SURVEY.md §8(c) — the golden fixtures are tie-free).
 * Parity pinned against tests/golden/real_env.npz (generated from the reference itself).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int ora_real_obs_size(int N, int M, int L) { return M * L + N * M * L + ((N * M) / 2) * L + M; }

/* variants: 0 RealConstellationEnv, 1 RealPowerConstellationEnv, 2 InterferenceConstellationEnv;
   the power variants append [power_i, power[top_n]] to every observation
   (real_power_constellation_env.py:226-229, :260-264) */
int ora_realx_obs_size(int variant, int N, int M, int L) {
    return ora_real_obs_size(N, M, L) + (variant > 0 ? N + 1 : 0);
}

/* beta[i][j][l] at time k (real_constellation_env.py:110 and :164-168) */
void ora_real_beta(const double *table, const double *prios, int n, int m, int T, int L, int k, double *beta) {
    int eff = T - k < L ? T - k : L;
    if (eff < 0) eff = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < m; ++j)
            for (int l = 0; l < L; ++l) {
                const double v = l < eff ? table[((int64_t)i * m + j) * T + k + l] : 0.0;
                beta[((int64_t)i * m + j) * L + l] = v * prios[j];
            }
}

static double row_total(const double *beta, int m, int L, int a, int j) {
    const double *p = beta + ((int64_t)a * m + j) * L;
    double s = p[0];
    for (int l = 1; l < L; ++l) s = s + p[l];
    return s;
}

/* key order helpers: descending value, ties -> lower index first */
static int before_desc(double va, int ia, double vb, int ib) { return va > vb || (va == vb && ia < ib); }

/* the `cnt` best indices of v[0..len) in descending stable order (selection, O(cnt*len)) */
static void top_desc(const double *v, int len, int cnt, int *out) {
    for (int c = 0; c < cnt; ++c) {
        int best = -1;
        for (int j = 0; j < len; ++j) {
            int used = 0;
            for (int q = 0; q < c; ++q) used |= out[q] == j;
            if (used) continue;
            if (best < 0 || before_desc(v[j], j, v[best], best)) best = j;
        }
        out[c] = best;
    }
}

/* observation rows of all agents (real_constellation_env.py:177-230); obs [n][obs_size];
   power != NULL: the power variants' trailing power observation */
void ora_realx_obs(const double *beta, int n, int m, int L, int N, int M, const int64_t *prev, const double *power,
                   int done, double *obs) {
    const int osz = ora_real_obs_size(N, M, L) + (power ? N + 1 : 0);
    if (done) {
        memset(obs, 0, sizeof(double) * (size_t)n * osz);
        return;
    }
    const int M2 = M / 2;
    double *tot = malloc(sizeof(double) * (size_t)n * m);
    double *best = malloc(sizeof(double) * (size_t)n);
    double *row = malloc(sizeof(double) * (size_t)m);
    int *top = malloc(sizeof(int) * (size_t)M), *topn = malloc(sizeof(int) * (size_t)N);
    int *oth = malloc(sizeof(int) * (size_t)(M2 > 0 ? M2 : 1));
    for (int a = 0; a < n; ++a)
        for (int j = 0; j < m; ++j) tot[(int64_t)a * m + j] = row_total(beta, m, L, a, j);
    for (int i = 0; i < n; ++i) {
        double *o = obs + (int64_t)i * osz;
        top_desc(tot + (int64_t)i * m, m, M, top);  /* np.argsort(-total_agent_benefits)[:M] */
        for (int k = 0; k < M; ++k)
            for (int l = 0; l < L; ++l) *o++ = beta[((int64_t)i * m + top[k]) * L + l];
        for (int a = 0; a < n; ++a) {  /* np.max(total_beta[:, top], axis=1) */
            double b = tot[(int64_t)a * m + top[0]];
            for (int k = 1; k < M; ++k) {
                const double v = tot[(int64_t)a * m + top[k]];
                b = v > b ? v : b;
            }
            best[a] = b;
        }
        best[i] = -INFINITY;
        top_desc(best, n, N, topn);  /* np.argsort(-best)[:N] */
        for (int a = 0; a < N; ++a)
            for (int k = 0; k < M; ++k)
                for (int l = 0; l < L; ++l) *o++ = beta[((int64_t)topn[a] * m + top[k]) * L + l];
        for (int a = 0; a < N; ++a) {
            /* np.argsort(row with top-M columns = -inf)[-M//2:]: the M//2 largest in
               ascending stable order -> pick descending with ties to the HIGHER index,
               then reverse */
            for (int j = 0; j < m; ++j) row[j] = tot[(int64_t)topn[a] * m + j];
            for (int k = 0; k < M; ++k) row[top[k]] = -INFINITY;
            for (int c = 0; c < M2; ++c) {
                int bj = -1;
                for (int j = 0; j < m; ++j) {
                    int used = 0;
                    for (int q = 0; q < c; ++q) used |= oth[q] == j;
                    if (used) continue;
                    if (bj < 0 || row[j] > row[bj] || (row[j] == row[bj] && j > bj)) bj = j;
                }
                oth[c] = bj;
            }
            for (int c = M2 - 1; c >= 0; --c)
                for (int l = 0; l < L; ++l) *o++ = beta[((int64_t)topn[a] * m + oth[c]) * L + l];
        }
        for (int k = 0; k < M; ++k) *o++ = top[k] == prev[i] ? 1.0 : 0.0;
        if (power) {
            *o++ = power[i];
            for (int a = 0; a < N; ++a) *o++ = power[topn[a]];
        }
    }
    free(tot);
    free(best);
    free(row);
    free(top);
    free(topn);
    free(oth);
}

void ora_real_obs(const double *beta, int n, int m, int L, int N, int M, const int64_t *prev, int done,
                  double *obs) {
    ora_realx_obs(beta, n, m, L, N, M, prev, NULL, done, obs);
}

/* reset (real_constellation_env.py:94-114, constant benefits): k = 0, prev = arange(n) */
void ora_real_reset(const double *table, const double *prios, int n, int m, int T, int L, int N, int M,
                    double *beta, int64_t *prev, double *obs) {
    ora_real_beta(table, prios, n, m, T, L, 0, beta);
    for (int i = 0; i < n; ++i) prev[i] = i;
    ora_real_obs(beta, n, m, L, N, M, prev, 0, obs);
}

/* step (real_constellation_env.py:135-175): beta / prev / *k advanced in place */
void ora_real_step(const double *table, const double *prios, const double *T_trans, int n, int m, int T, int L,
                   int N, int M, double lambda, int *k, double *beta, int64_t *prev, const int64_t *actions,
                   double *rewards, int *done, double *obs) {
    double *cnt = calloc((size_t)m, sizeof(double));
    for (int i = 0; i < n; ++i) cnt[actions[i]] += 1.0;
    for (int i = 0; i < n; ++i) {
        const int c = (int)actions[i];
        const double cond = row_total(beta, m, L, i, c) > 1e-12 ? 1.0 : 0.0;
        const double pen = T_trans[(int64_t)prev[i] * m + c] * cond;
        const double bh = beta[((int64_t)i * m + c) * L] - lambda * pen;
        rewards[i] = bh > 0 ? bh / cnt[c] : bh;
    }
    free(cnt);
    *k += 1;
    *done = *k >= T;
    ora_real_beta(table, prios, n, m, T, L, *k, beta);
    for (int i = 0; i < n; ++i) prev[i] = actions[i];
    ora_real_obs(beta, n, m, L, N, M, prev, *done, obs);
}

/* ---- power / interference variants ----------------------------- */

/* reset of the power variants (real_power_constellation_env.py:118-135,
   interference_constellation_env.py:147-169, constant setup): prev_assigns given (the
   reference draws np.random.choice(m, n, replace=False) from numpy's global stream),
   power_states = 1 */
void ora_realx_reset(int variant, const double *table, const double *prios, int n, int m, int T, int L, int N, int M,
                     const int64_t *prev0, double *beta, int64_t *prev, double *power, double *obs) {
    ora_real_beta(table, prios, n, m, T, L, 0, beta);
    for (int i = 0; i < n; ++i) {
        prev[i] = variant > 0 ? prev0[i] : i;
        power[i] = 1.0;
    }
    ora_realx_obs(beta, n, m, L, N, M, prev, variant > 0 ? power : NULL, 0, obs);
}

/* step of the three variants.  variant 1 (real_power_constellation_env.py:137-191): the
   RealConstellationEnv reward with beta_hat zeroed for agents below 1e-12 power and 0 for
   dead agents; variant 2 (interference_constellation_env.py:171-205, :309-353): reward =
   beta[i, a_i, 0] * 0.5 ** conflicts, where conflicts = sum over agents of the same
   frequency band of neighbor_matrix[a_i, a_j] * applicable_j - 1, split over the
   applicable agents on the task, minus lambda on a handover.  Both then update power. */
void ora_realx_step(int variant, const double *table, const double *prios, const double *T_trans, const int *bands,
                    const double *nbr, int n, int m, int T, int L, int N, int M, double lambda, int *k, double *beta,
                    int64_t *prev, double *power, const int64_t *actions, double *rewards, int *done, double *obs) {
    if (variant == 0) {
        ora_real_step(table, prios, T_trans, n, m, T, L, N, M, lambda, k, beta, prev, actions, rewards, done, obs);
        return;
    }
    double *cnt = calloc((size_t)m, sizeof(double));
    int *app = calloc((size_t)n, sizeof(int));
    if (variant == 1) {
        for (int i = 0; i < n; ++i) cnt[actions[i]] += 1.0;
        for (int i = 0; i < n; ++i) {
            if (!(power[i] > 0)) {
                rewards[i] = 0.0;
                continue;
            }
            const int c = (int)actions[i];
            double bh;
            if (power[i] < 1e-12) {
                bh = 0.0;
            } else {
                const double cond = row_total(beta, m, L, i, c) > 1e-12 ? 1.0 : 0.0;
                const double pen = T_trans[(int64_t)prev[i] * m + c] * cond;
                bh = beta[((int64_t)i * m + c) * L] - lambda * pen;
            }
            rewards[i] = bh > 0 ? bh / cnt[c] : bh;
        }
    } else {
        for (int i = 0; i < n; ++i) {
            const int alive = power[i] <= 0 ? 0 : 1;
            const int meaningful = beta[((int64_t)i * m + actions[i]) * L] < 1e-12 ? 0 : 1;
            app[i] = alive * meaningful;
            if (app[i]) cnt[actions[i]] += 1.0;
        }
        for (int i = 0; i < n; ++i) {
            const int c = (int)actions[i];
            double conf = 0.0;
            for (int a = 0; a < n; ++a)
                if (bands[a] == bands[i]) conf = conf + nbr[(int64_t)c * m + actions[a]] * (double)app[a];
            conf = conf - 1.0;
            double r = beta[((int64_t)i * m + c) * L] * pow(0.5, conf);
            if (cnt[c] > 0) r = r / cnt[c];
            if (app[i] && prev[i] != c) r = r - lambda;
            rewards[i] = r;
        }
    }
    *k += 1;
    *done = *k >= T;
    for (int i = 0; i < n; ++i) {  /* power update on the pre-step beta */
        if (power[i] > 0) {
            if (beta[((int64_t)i * m + actions[i]) * L] > 1e-12) {
                power[i] -= 0.2;
            } else {
                const double p = power[i] + 0.1;
                power[i] = p < 1.0 ? p : 1.0;
            }
        }
    }
    free(cnt);
    free(app);
    ora_real_beta(table, prios, n, m, T, L, *k, beta);
    for (int i = 0; i < n; ++i) prev[i] = actions[i];
    ora_realx_obs(beta, n, m, L, N, M, prev, power, *done, obs);
}
