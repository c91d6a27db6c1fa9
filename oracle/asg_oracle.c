/*
 * asg_oracle.c -- CPU ORACLE for the sequential-assignment env hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (marl_sap_amd/, include/) links,
 * loads or calls this file.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / the timed CPU baseline.
 *
 * It is a plain-C restatement of the reference algorithm, pinned against the golden
 * vectors in tests/golden/ (generated from the reference itself by
 * tests/golden/make_golden.py).  Every function cites the reference line it follows.
 *
 *   - legacy MT19937 stream of numpy's global RandomState (SURVEY.md Appendix A;
 *     third-party: numpy 2.2.6 `RandomState`, consumed by
 *     src/envs/mock_constellation_env.py:276-299 and :105)
 *   - generate_benefits_over_time           mock_constellation_env.py:276-299
 *   - MockConstellationEnv.reset             mock_constellation_env.py:94-114
 *   - MockConstellationEnv.step              mock_constellation_env.py:116-162
 *   - MockConstellationEnv.beta_hat          mock_constellation_env.py:228-274
 *   - scipy.optimize.linear_sum_assignment   third-party (scipy 1.15.3,
 *     rectangular LSAP, shortest augmenting path); restated from its published
 *     algorithm; call sites mock_constellation_env.py:122,
 *     sap_selectors.py:32,90, non_rl_selectors.py:47
 *
 * Build: oracle/Makefile  ->  oracle/libasg_oracle.so  (gcc, -ffp-contract=off so that
 * every double operation rounds exactly like numpy's scalar arithmetic).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------ */
/* legacy MT19937 (numpy RandomState)                                              */
/* ------------------------------------------------------------------------------ */
#define MT_N 624
#define MT_M 397

typedef struct {
    uint32_t key[MT_N];
    int pos;
    uint64_t drawn; /* words consumed since seeding */
} ora_mt;

/* np.random.seed(s) with an int seed: Knuth init_genrand */
void ora_mt_seed(ora_mt *st, uint32_t seed) {
    st->key[0] = seed;
    for (int i = 1; i < MT_N; i++) {
        uint32_t p = st->key[i - 1];
        st->key[i] = 1812433253u * (p ^ (p >> 30)) + (uint32_t)i;
    }
    st->pos = MT_N;
    st->drawn = 0;
}

static void mt_twist(ora_mt *st) {
    uint32_t *k = st->key;
    for (int i = 0; i < MT_N; i++) {
        uint32_t y = (k[i] & 0x80000000u) | (k[(i + 1) % MT_N] & 0x7fffffffu);
        uint32_t v = k[(i + MT_M) % MT_N] ^ (y >> 1);
        if (y & 1u) v ^= 0x9908b0dfu;
        k[i] = v;
    }
    st->pos = 0;
}

uint32_t ora_mt_next(ora_mt *st) {
    if (st->pos >= MT_N) mt_twist(st);
    st->drawn++;
    uint32_t y = st->key[st->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

/* RandomState.random_sample / rand(): 53-bit double from two words */
double ora_mt_double(ora_mt *st) {
    int32_t a = (int32_t)(ora_mt_next(st) >> 5);
    int32_t b = (int32_t)(ora_mt_next(st) >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

/* RandomState.uniform(lo, hi) = lo + (hi - lo) * next_double */
double ora_mt_uniform(ora_mt *st, double lo, double hi) {
    double range = hi - lo;
    return lo + range * ora_mt_double(st);
}

/* bounded draw used by legacy shuffle: masked rejection on 32-bit words */
static uint32_t mt_interval(ora_mt *st, uint32_t max) {
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
    mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (ora_mt_next(st) & mask)) > max) {}
    return v;
}

/* RandomState.permutation(m): arange + Fisher-Yates from the top */
void ora_mt_permutation(ora_mt *st, int m, int64_t *out) {
    for (int i = 0; i < m; i++) out[i] = i;
    for (int i = m - 1; i >= 1; i--) {
        uint32_t j = mt_interval(st, (uint32_t)i);
        int64_t t = out[i]; out[i] = out[j]; out[j] = t;
    }
}

/* RandomState.choice([1,1,1,10]): one word masked to 2 bits (randint(0,4)) */
static int mt_choice_scale(ora_mt *st) {
    static const int pool[4] = {1, 1, 1, 10};
    return pool[ora_mt_next(st) & 3u];
}

void ora_mt_get_state(const ora_mt *st, uint32_t *key, int *pos) {
    memcpy(key, st->key, sizeof(st->key));
    *pos = st->pos;
}

/* ------------------------------------------------------------------------------ */
/* benefit tables: generate_benefits_over_time (mock_constellation_env.py:276-299) */
/* ------------------------------------------------------------------------------ */
/* np.log(0.05) as numpy rounds it: -0x1.7f7427b73e391p+1 */
static const double LOG_005 = -0x1.7f7427b73e391p+1;

/* out: [n][m][T] row-major (numpy layout of the reference table) */
void ora_generate(ora_mt *st, int n, int m, int T, double wmin, double wmax, double *out) {
    memset(out, 0, sizeof(double) * (size_t)n * m * T);
    for (int j = 0; j < m; j++) {                          /* :281 task loop outer */
        int scale = mt_choice_scale(st);                   /* :282 */
        for (int i = 0; i < n; i++) {                      /* :283 */
            double r = ora_mt_double(st);                  /* :285 rand() > 0.75 */
            if (!(r > 0.75)) continue;
            double center = ora_mt_uniform(st, 0.0, (double)T);     /* :289 */
            double spread = ora_mt_uniform(st, wmin, wmax);         /* :292 */
            /* CPython float ** 2 is libm pow(x, 2.0), which can differ from x*x by 1 ulp */
            double s2 = sqrt(pow(spread, 2.0) / -8.0 / LOG_005);    /* :293 */
            for (int t = 0; t < T; t++) {                           /* :296-298 */
                double q = -pow((double)t - center, 2.0) / s2 / 2.0;
                out[((size_t)i * m + j) * T + t] = (double)scale * exp(q);
            }
        }
    }
}

/* ------------------------------------------------------------------------------ */
/* beta_hat (mock_constellation_env.py:228-274), one time slice                    */
/* ------------------------------------------------------------------------------ */
/* T_trans may be NULL (default 1 - I, :40).  out[i][j] = beta - lambda*pen */
void ora_beta_hat(const double *beta, const int64_t *prev, int n, int m,
                  const double *T_trans, double lambda, double *out) {
    for (int i = 0; i < n; i++) {
        int64_t p = prev[i];
        for (int j = 0; j < m; j++) {
            /* (onehot(prev) @ T_trans)[i, j] = T_trans[p, j]  (:250-260) */
            double tt = T_trans ? T_trans[(size_t)p * m + j] : (j == p ? 0.0 : 1.0);
            double b = beta[(size_t)i * m + j];
            double pen = tt * (b > 1e-12 ? 1.0 : 0.0);              /* :263-266 */
            out[(size_t)i * m + j] = b - lambda * pen;              /* :269-270 */
        }
    }
}

/* ------------------------------------------------------------------------------ */
/* scipy linear_sum_assignment restatement                  */
/* ------------------------------------------------------------------------------ */
/* inner-loop iterations of the last ora_lsa call (instrumentation for tuning) */
static long g_lsa_iters;
long ora_lsa_iterations(void) { return g_lsa_iters; }

/* returns 0 ok, -1 invalid entries (NaN / -inf after sign), -2 infeasible.
 * row/col receive min(nr, nc) entries. */
int ora_lsa(const double *C_in, int nr0, int nc0, int maximize, int64_t *row_out, int64_t *col_out) {
    if (nr0 == 0 || nc0 == 0) return 0;
    int transpose = nc0 < nr0;
    int nr = transpose ? nc0 : nr0, nc = transpose ? nr0 : nc0;
    double *C = (double *)malloc(sizeof(double) * (size_t)nr * nc);
    for (int i = 0; i < nr0; i++)
        for (int j = 0; j < nc0; j++) {
            double v = C_in[(size_t)i * nc0 + j];
            if (transpose) C[(size_t)j * nr0 + i] = v; else C[(size_t)i * nc0 + j] = v;
        }
    if (maximize)
        for (size_t k = 0; k < (size_t)nr * nc; k++) C[k] = -C[k];
    for (size_t k = 0; k < (size_t)nr * nc; k++)
        if (C[k] != C[k] || C[k] == -INFINITY) { free(C); return -1; }

    double *u = calloc(nr, sizeof(double)), *v = calloc(nc, sizeof(double));
    double *spc = malloc(sizeof(double) * nc);
    int64_t *path = malloc(sizeof(int64_t) * nc), *col4row = malloc(sizeof(int64_t) * nr);
    int64_t *row4col = malloc(sizeof(int64_t) * nc), *remaining = malloc(sizeof(int64_t) * nc);
    char *SR = malloc(nr), *SC = malloc(nc);
    for (int i = 0; i < nr; i++) col4row[i] = -1;
    for (int j = 0; j < nc; j++) { row4col[j] = -1; path[j] = -1; }
    int status = 0;
    g_lsa_iters = 0;

    for (int cur = 0; cur < nr; cur++) {
        double minv = 0.0;
        int nrem = nc;
        for (int it = 0; it < nc; it++) remaining[it] = nc - it - 1;
        memset(SR, 0, nr); memset(SC, 0, nc);
        for (int j = 0; j < nc; j++) spc[j] = INFINITY;
        int64_t i = cur, sink = -1;
        while (sink == -1) {
            g_lsa_iters++;
            int64_t index = -1;
            double lowest = INFINITY;
            SR[i] = 1;
            for (int it = 0; it < nrem; it++) {
                int64_t j = remaining[it];
                double r = minv + C[(size_t)i * nc + j] - u[i] - v[j];
                if (r < spc[j]) { path[j] = i; spc[j] = r; }
                if (spc[j] < lowest || (spc[j] == lowest && row4col[j] == -1)) {
                    lowest = spc[j]; index = it;
                }
            }
            minv = lowest;
            if (minv == INFINITY) { status = -2; goto done; }
            int64_t j = remaining[index];
            if (row4col[j] == -1) sink = j; else i = row4col[j];
            SC[j] = 1;
            remaining[index] = remaining[--nrem];
        }
        u[cur] += minv;
        for (int r = 0; r < nr; r++)
            if (SR[r] && r != cur) u[r] += minv - spc[col4row[r]];
        for (int c = 0; c < nc; c++)
            if (SC[c]) v[c] -= minv - spc[c];
        for (int64_t j = sink;;) {
            int64_t pi = path[j];
            row4col[j] = pi;
            int64_t t = col4row[pi]; col4row[pi] = j; j = t;
            if (pi == cur) break;
        }
    }
    if (transpose) {
        /* (col4row[argsort(col4row)], argsort(col4row)); col4row is a permutation
         * of distinct ids, so argsort is unambiguous */
        int k;
        int64_t *order = malloc(sizeof(int64_t) * nr);
        for (int a = 0; a < nr; a++) order[a] = a;
        for (int a = 1; a < nr; a++) {                   /* insertion sort by value */
            int64_t key = order[a]; int b = a - 1;
            while (b >= 0 && col4row[order[b]] > col4row[key]) { order[b + 1] = order[b]; b--; }
            order[b + 1] = key;
        }
        for (k = 0; k < nr; k++) { row_out[k] = col4row[order[k]]; col_out[k] = order[k]; }
        free(order);
    } else {
        for (int r = 0; r < nr; r++) { row_out[r] = r; col_out[r] = col4row[r]; }
    }
done:
    free(C); free(u); free(v); free(spc); free(path); free(col4row); free(row4col);
    free(remaining); free(SR); free(SC);
    return status;
}

/* ------------------------------------------------------------------------------ */
/* MockConstellationEnv                                                            */
/* ------------------------------------------------------------------------------ */
/* obs for step k: [onehot(assign) | table[:,:,k] | ... | table[:,:,k+L-1]] with zero
 * blocks past T (mock_constellation_env.py:107-112, :147-152).  assign may be NULL
 * (reset: all-zero curr_assignment, :96/:107). obs: [n][m*(L+1)] */
static void build_obs(const double *table, int n, int m, int T, int L, int k,
                      const int64_t *assign, double *obs) {
    int W = m * (L + 1);
    for (int i = 0; i < n; i++) {
        double *o = obs + (size_t)i * W;
        for (int j = 0; j < m; j++) o[j] = (assign && assign[i] == j) ? 1.0 : 0.0;
        for (int l = 0; l < L; l++)
            for (int j = 0; j < m; j++)
                o[m * (l + 1) + j] = (k + l < T) ? table[((size_t)i * m + j) * T + k + l] : 0.0;
    }
}

/* construct (with generated table when table_injected == 0, :32-34) then reset
 * (:94-114). table: [n][m][T] in/out.  Returns -1 if m < n (choice without
 * replacement raises in the reference, :105). */
int ora_env_construct_reset(ora_mt *st, int n, int m, int T, int L, int table_injected,
                            double *init_table, double *table, int64_t *prev_assigns,
                            double *obs, double *beta) {
    if (!table_injected) {
        ora_generate(st, n, m, T, 5.0, 8.0, init_table);   /* __init__ :34 */
        ora_generate(st, n, m, T, 3.0, 6.0, table);        /* reset :100 */
    }
    if (n > m) return -1;
    int64_t *perm = malloc(sizeof(int64_t) * m);
    ora_mt_permutation(st, m, perm);                       /* :105 choice(m,n,False) */
    memcpy(prev_assigns, perm, sizeof(int64_t) * n);
    free(perm);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < m; j++) beta[(size_t)i * m + j] = table[((size_t)i * m + j) * T];
    build_obs(table, n, m, T, L, 0, NULL, obs);
    return 0;
}

/* reset of an env that already exists (second and later episodes, :94-114) */
int ora_env_reset(ora_mt *st, int n, int m, int T, int L, int table_injected, double *table,
                  int64_t *prev_assigns, double *obs, double *beta) {
    if (!table_injected) ora_generate(st, n, m, T, 3.0, 6.0, table);
    if (n > m) return -1;
    int64_t *perm = malloc(sizeof(int64_t) * m);
    ora_mt_permutation(st, m, perm);
    memcpy(prev_assigns, perm, sizeof(int64_t) * n);
    free(perm);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < m; j++) beta[(size_t)i * m + j] = table[((size_t)i * m + j) * T];
    build_obs(table, n, m, T, L, 0, NULL, obs);
    return 0;
}

/* step (:116-162).  k: in/out step counter.  beta: in (current) / out (next).
 * prev_assigns: in/out.  Exactly one of actions (int64 [n]) and bids (double [n][m],
 * bids_as_actions, :121-122) is non-NULL.  rewards out double [n]. returns done, or
 * a negative LSA status when the bids are invalid. */
int ora_env_step(int n, int m, int T, int L, double lambda, const double *table,
                 const double *T_trans, int *k, double *beta, int64_t *prev_assigns,
                 const int64_t *actions, const double *bids, double *rewards, double *obs) {
    int64_t *a = malloc(sizeof(int64_t) * n);
    if (bids) {
        int64_t *rows = malloc(sizeof(int64_t) * n);
        int st = ora_lsa(bids, n, m, 1, rows, a);
        free(rows);
        if (st) { free(a); return st; }
    } else {
        memcpy(a, actions, sizeof(int64_t) * n);
    }
    double *bh = malloc(sizeof(double) * (size_t)n * m);
    ora_beta_hat(beta, prev_assigns, n, m, T_trans, lambda, bh);   /* :126 */
    double *cnt = calloc(m, sizeof(double));
    for (int i = 0; i < n; i++) cnt[a[i]] += 1.0;                   /* :128-130 */
    for (int i = 0; i < n; i++) {                                  /* :132-138 */
        double b = bh[(size_t)i * m + a[i]];
        rewards[i] = (b > 0) ? b / cnt[a[i]] : b;
    }
    *k += 1;                                                       /* :145 */
    build_obs(table, n, m, T, L, *k, a, obs);                      /* :147-152 */
    int done = *k >= T;                                            /* :154 */
    for (int i = 0; i < n; i++)
        for (int j = 0; j < m; j++)
            beta[(size_t)i * m + j] = done ? 0.0 : table[((size_t)i * m + j) * T + *k];
    memcpy(prev_assigns, a, sizeof(int64_t) * n);                  /* :160 */
    free(a); free(bh); free(cnt);
    return done;
}

size_t ora_mt_sizeof(void) { return sizeof(ora_mt); }
uint64_t ora_mt_drawn(const ora_mt *st) { return st->drawn; }
