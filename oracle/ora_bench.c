/*
 * ora_bench.c -- TEST INFRASTRUCTURE ONLY: the CPU baseline of bench.py.
 *
 * Times the scalar C restatement (mas_oracle.c) the way SURVEY.md 8(d) asks
 * for the reference's CPU path: uniform-random actions over
 * MultiDiscrete([3,3,3,2,2,2]) (demo.py's random policy, demo.py:119,135-141),
 * auto-reset on done, envs partitioned over `threads` POSIX threads, each
 * thread stepping its envs round-robin until `budget_s` seconds pass.  No
 * ctypes call per step: the whole loop runs in C.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mas_oracle.h"

typedef struct {
    const mas_config* cfg;
    const uint64_t* seeds6;  /* [n_envs][6] PCG64 states of this thread's envs */
    int64_t n_envs;
    double budget_s;
    uint64_t act_seed;
    int64_t env_steps;       /* out */
    double seconds;          /* out */
    int failed;              /* out */
} job;

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static uint64_t splitmix(uint64_t* s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static void* run_job(void* arg)
{
    job* j = (job*)arg;
    const int A = j->cfg->n_agents;
    char err[256];
    ora_env** envs = (ora_env**)calloc((size_t)j->n_envs, sizeof(ora_env*));
    int D = 0;
    for (int64_t e = 0; e < j->n_envs; ++e) {
        envs[e] = ora_env_create(j->cfg, err, (int)sizeof(err));
        if (!envs[e]) { j->failed = 1; break; }
        ora_env_set_rng(envs[e], j->seeds6 + 6 * e);
        D = ora_env_obs_dim(envs[e]);
    }
    float* obs = (float*)malloc(sizeof(float) * (size_t)A * (size_t)(D > 0 ? D : 1));
    float rew[64];
    int8_t act[64 * 6];
    if (!j->failed) {
        for (int64_t e = 0; e < j->n_envs; ++e) ora_env_reset(envs[e], obs);
        static const int hi[6] = {3, 3, 3, 2, 2, 2};
        uint64_t rs = j->act_seed;
        int64_t steps = 0;
        const double t0 = now_s();
        double t = t0;
        while (t - t0 < j->budget_s) {
            for (int64_t e = 0; e < j->n_envs; ++e) {
                for (int k = 0; k < A * 6; ++k) act[k] = (int8_t)(splitmix(&rs) % (uint64_t)hi[k % 6]);
                if (ora_env_step(envs[e], act, obs, rew)) ora_env_reset(envs[e], obs);
            }
            steps += j->n_envs;
            t = now_s();
        }
        j->env_steps = steps;
        j->seconds = t - t0;
    }
    for (int64_t e = 0; e < j->n_envs; ++e)
        if (envs[e]) ora_env_destroy(envs[e]);
    free(envs);
    free(obs);
    return NULL;
}

/* Steps n_envs envs (PCG64 states seeds6 [n_envs][6]) on `threads` threads
 * for about budget_s seconds.  out[0] = env-steps done, out[1] = wall seconds
 * (the slowest thread).  Returns 0, or -1 if an env could not be created. */
int32_t ora_bench_run(const mas_config* cfg, const uint64_t* seeds6, int64_t n_envs, int32_t threads,
                      double budget_s, double* out)
{
    if (threads < 1) threads = 1;
    if (threads > n_envs) threads = (int32_t)n_envs;
    job* jobs = (job*)calloc((size_t)threads, sizeof(job));
    pthread_t* tid = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    int64_t lo = 0;
    for (int k = 0; k < threads; ++k) {
        const int64_t hi = n_envs * (k + 1) / threads;
        jobs[k].cfg = cfg;
        jobs[k].seeds6 = seeds6 + 6 * lo;
        jobs[k].n_envs = hi - lo;
        jobs[k].budget_s = budget_s;
        jobs[k].act_seed = 0x1234567ULL + (uint64_t)k;
        lo = hi;
        pthread_create(&tid[k], NULL, run_job, &jobs[k]);
    }
    int64_t steps = 0;
    double secs = 0.0;
    int failed = 0;
    for (int k = 0; k < threads; ++k) {
        pthread_join(tid[k], NULL);
        steps += jobs[k].env_steps;
        if (jobs[k].seconds > secs) secs = jobs[k].seconds;
        failed |= jobs[k].failed;
    }
    free(jobs);
    free(tid);
    out[0] = (double)steps;
    out[1] = secs;
    return failed ? -1 : 0;
}
