/*
 * asg_rollout.c -- multi-threaded CPU rollout built on the oracle env (TEST / BASELINE
 * INFRASTRUCTURE ONLY; see asg_oracle.c).  bench.py's cpu_baseline leg times it as the
 * "strong" CPU number next to the Python ParallelRunner-protocol port
 * (oracle/cpu_parallel_runner.py).  Each env owns a legacy-MT19937 stream seeded
 * (seed + global env index), runs construct+reset (mock_constellation_env.py:17-114)
 * and T steps (:116-162) under a uniform random policy, exactly as the reference env
 * would for that stream.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct { uint32_t key[624]; int pos; uint64_t drawn; } ora_mt;
void ora_mt_seed(ora_mt *st, uint32_t seed);
uint32_t ora_mt_next(ora_mt *st);
int ora_env_construct_reset(ora_mt *st, int n, int m, int T, int L, int table_injected,
                            double *init_table, double *table, int64_t *prev_assigns,
                            double *obs, double *beta);
int ora_env_reset(ora_mt *st, int n, int m, int T, int L, int table_injected, double *table,
                  int64_t *prev_assigns, double *obs, double *beta);
int ora_env_step(int n, int m, int T, int L, double lambda, const double *table,
                 const double *T_trans, int *k, double *beta, int64_t *prev_assigns,
                 const int64_t *actions, const double *bids, double *rewards, double *obs);

typedef struct {
    int e0, e1, n, m, T, L, episodes;
    double lambda;
    uint32_t seed;
    double *returns;
} job_t;

static void *worker(void *p) {
    job_t *J = (job_t *)p;
    int n = J->n, m = J->m, T = J->T, L = J->L;
    double *init = malloc(sizeof(double) * (size_t)n * m * T);
    double *table = malloc(sizeof(double) * (size_t)n * m * T);
    double *obs = malloc(sizeof(double) * (size_t)n * m * (L + 1));
    double *beta = malloc(sizeof(double) * (size_t)n * m);
    double *rew = malloc(sizeof(double) * n);
    int64_t *prev = malloc(sizeof(int64_t) * n), *act = malloc(sizeof(int64_t) * n);
    ora_mt st;
    for (int e = J->e0; e < J->e1; e++) {
        ora_mt_seed(&st, J->seed + (uint32_t)e);
        double ret = 0.0;
        for (int ep = 0; ep < J->episodes; ep++) {
            if (ep == 0) ora_env_construct_reset(&st, n, m, T, L, 0, init, table, prev, obs, beta);
            else ora_env_reset(&st, n, m, T, L, 0, table, prev, obs, beta);
            int k = 0;
            ret = 0.0;
            for (int t = 0; t < T; t++) {
                for (int i = 0; i < n; i++) act[i] = ora_mt_next(&st) % (uint32_t)m;
                ora_env_step(n, m, T, L, J->lambda, table, NULL, &k, beta, prev, act, NULL, rew, obs);
                for (int i = 0; i < n; i++) ret += rew[i];
            }
        }
        J->returns[e] = ret;
    }
    free(init); free(table); free(obs); free(beta); free(rew); free(prev); free(act);
    return NULL;
}

/* Runs `episodes` episodes on each of E envs with `threads` threads; returns the
 * wall time in seconds; returns_out[E] receives the last episode's return. */
double ora_rollout_random(int E, int n, int m, int T, int L, double lambda, uint32_t seed,
                          int threads, int episodes, double *returns_out) {
    if (threads < 1) threads = 1;
    if (threads > E) threads = E;
    pthread_t *th = malloc(sizeof(pthread_t) * threads);
    job_t *jobs = malloc(sizeof(job_t) * threads);
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job_t){E * t / threads, E * (t + 1) / threads, n, m, T, L, episodes, lambda,
                          seed, returns_out};
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    free(th); free(jobs);
    return (b.tv_sec - a.tv_sec) + 1e-9 * (b.tv_nsec - a.tv_nsec);
}
