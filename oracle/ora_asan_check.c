/*
 * ora_asan_check.c -- TEST INFRASTRUCTURE ONLY: drives the oracle under
 * AddressSanitizer + UndefinedBehaviorSanitizer (`make asan`).
 *
 * usage: ora_asan_check <mas_config blob> <envs> <steps> <threads>
 * The blob is the raw bytes of a mas_config (include/masurvival.h) written by
 * tests/test_oracle_sanitize.py from masurvival.config.ResolvedConfig.  Runs
 * random-action episodes with auto-reset through ora_bench_run (threads) and
 * then a single-thread pass of reset/step/flush_stats/debug on one env.
 */
#include <stdio.h>
#include <stdlib.h>

#include "mas_oracle.h"

int32_t ora_bench_run(const mas_config* cfg, const uint64_t* seeds6, int64_t n_envs, int32_t threads,
                      double budget_s, double* out);

int main(int argc, char** argv)
{
    if (argc != 5) {
        fprintf(stderr, "usage: %s cfg.bin envs steps threads\n", argv[0]);
        return 2;
    }
    mas_config cfg;
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(&cfg, sizeof(cfg), 1, f) != 1) {
        fprintf(stderr, "cannot read %s (%zu bytes expected)\n", argv[1], sizeof(cfg));
        return 2;
    }
    fclose(f);
    const int64_t n = atoll(argv[2]);
    const int steps = atoi(argv[3]);
    const int threads = atoi(argv[4]);
    uint64_t* seeds = (uint64_t*)calloc((size_t)(6 * n), sizeof(uint64_t));
    for (int64_t e = 0; e < n; ++e) {
        /* any valid PCG64 state: odd increment */
        seeds[6 * e + 0] = 0x243F6A8885A308D3ULL ^ (uint64_t)e;
        seeds[6 * e + 1] = 0x13198A2E03707344ULL + 7ULL * (uint64_t)e;
        seeds[6 * e + 2] = 0xA4093822299F31D0ULL;
        seeds[6 * e + 3] = 0x082EFA98EC4E6C89ULL | 1ULL;
    }
    double out[2];
    if (ora_bench_run(&cfg, seeds, n, threads, 0.5, out) != 0) {
        fprintf(stderr, "ora_bench_run failed\n");
        return 1;
    }
    char err[256];
    ora_env* e = ora_env_create(&cfg, err, (int)sizeof(err));
    if (!e) {
        fprintf(stderr, "create: %s\n", err);
        return 1;
    }
    ora_env_set_rng(e, seeds);
    const int A = cfg.n_agents, D = ora_env_obs_dim(e);
    float* obs = (float*)malloc(sizeof(float) * (size_t)(A * D));
    float rew[64], stats[MAS_STATS_WIDTH], dbg[512];
    int8_t act[64 * 6];
    uint64_t s = 1;
    ora_env_reset(e, obs);
    for (int t = 0; t < steps; ++t) {
        for (int k = 0; k < A * 6; ++k) {
            s = s * 6364136223846793005ULL + 1442695040888963407ULL;
            act[k] = (int8_t)((s >> 33) % (k % 6 < 3 ? 3u : 2u));
        }
        if (ora_env_step(e, act, obs, rew)) ora_env_reset(e, obs);
    }
    ora_env_flush_stats(e, stats);
    ora_env_debug(e, dbg, 512);
    ora_env_destroy(e);
    free(obs);
    free(seeds);
    printf("ok %.0f env-steps\n", out[0]);
    return 0;
}
