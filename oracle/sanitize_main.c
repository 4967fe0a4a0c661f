/* Sanitizer driver for the CPU oracle (test infrastructure only): random
 * swarms through every oracle entry point -- the batched solve on a thread
 * pool (TSan: the pool's shared state), the single-swarm solve with tables,
 * the CBAA with margins, LSAP / Hungarian -- and basic invariants (every
 * P_out a permutation). Built by `make -C oracle asan` / `make -C oracle
 * tsan`; tests/test_oracle_sanitize.py runs both. Exit 0 = clean run. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "aclswarm_oracle.h"

static unsigned long long rng = 88172645463325252ull;
static double urand(void) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (double)(rng >> 11) * (1.0 / 9007199254740992.0);
}

static int is_perm(int n, const uint16_t* P) {
  unsigned char seen[512];
  memset(seen, 0, sizeof(seen));
  for (int i = 0; i < n; ++i) {
    if (P[i] >= n || seen[P[i]]) return 0;
    seen[P[i]] = 1;
  }
  return 1;
}

static void swarm(int n, int F, int B, double* p, uint8_t* adj, double* gains, int32_t* fidx,
                  double* q, double* vel, uint16_t* P_in) {
  for (int f = 0; f < F; ++f) {
    for (int i = 0; i < n; ++i) {
      p[(f * n + i) * 3 + 0] = 20.0 * urand() - 10.0;
      p[(f * n + i) * 3 + 1] = 20.0 * urand() - 10.0;
      p[(f * n + i) * 3 + 2] = 2.0 * urand();
    }
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        const int e = (i != j) && (urand() < 0.8 || j == (i + 1) % n || i == (j + 1) % n);
        adj[((size_t)f * n + i) * n + j] = (uint8_t)e;
      }
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j)
        adj[((size_t)f * n + j) * n + i] = adj[((size_t)f * n + i) * n + j];
    for (size_t k = 0; k < (size_t)9 * n * n; ++k) gains[(size_t)f * 9 * n * n + k] = 0.1 * urand() - 0.05;
  }
  for (int b = 0; b < B; ++b) {
    fidx[b] = b % F;
    for (int i = 0; i < n; ++i) {
      q[(b * n + i) * 3 + 0] = 24.0 * urand() - 12.0;
      q[(b * n + i) * 3 + 1] = 24.0 * urand() - 12.0;
      q[(b * n + i) * 3 + 2] = 1.0 + urand();
      for (int k = 0; k < 3; ++k) vel[(b * n + i) * 3 + k] = 0.2 * urand() - 0.1;
      P_in[b * n + i] = (uint16_t)i;
    }
    for (int i = n - 1; i > 0; --i) {  // a random P_in for odd swarms
      if (!(b & 1)) break;
      const int j = (int)(urand() * (i + 1));
      const uint16_t t = P_in[b * n + i];
      P_in[b * n + i] = P_in[b * n + j];
      P_in[b * n + j] = t;
    }
  }
}

int main(void) {
  const acl_cntrl_gains_t g = {0.1, 0.1, 0.5, 0.3, 0.3, 0.1, 1.5, 0.5};
  const acl_safety_params_t s = {0.5, 0.3, 1.5, 1.2};
  int bad = 0;
  const int cases[][3] = {{6, 2, 16}, {20, 3, 24}, {37, 2, 8}, {70, 1, 4}};
  for (unsigned c = 0; c < sizeof(cases) / sizeof(cases[0]); ++c) {
    const int n = cases[c][0], F = cases[c][1], B = cases[c][2];
    double* p = malloc(sizeof(double) * F * n * 3);
    uint8_t* adj = malloc((size_t)F * n * n);
    double* gains = malloc(sizeof(double) * (size_t)F * 9 * n * n);
    int32_t* fidx = malloc(sizeof(int32_t) * B);
    double* q = malloc(sizeof(double) * B * n * 3);
    double* vel = malloc(sizeof(double) * B * n * 3);
    uint16_t* P_in = malloc(sizeof(uint16_t) * B * n);
    uint16_t* P_out = malloc(sizeof(uint16_t) * B * n);
    acl_swarm_status_t* st = malloc(sizeof(acl_swarm_status_t) * B);
    double* u = malloc(sizeof(double) * B * n * 3);
    double* us = malloc(sizeof(double) * B * n * 3);
    uint8_t* ca = malloc((size_t)B * n);
    uint16_t* who = malloc(sizeof(uint16_t) * n * n);
    swarm(n, F, B, p, adj, gains, fidx, q, vel, P_in);
    /* the thread pool, with and without margins, both schedules */
    for (int mode = 0; mode < 4; ++mode) {
      orc_solve_batch(B, n, 4, fidx, q, vel, p, adj, gains, P_in, &g, &s, mode & 1, P_out, st, u,
                      us, ca, mode >> 1);
      for (int b = 0; b < B; ++b) bad += !is_perm(n, P_out + b * n);
    }
    /* one swarm with its tables and gate margin */
    double gm = 0.0;
    orc_solve_g(n, q, vel, p, adj, gains, P_in, &g, &s, 1, P_out, st, u, us, ca, who, &gm);
    bad += !is_perm(n, P_out);
    /* the centralized comparator */
    double cost[2], Rt[6];
    uint16_t Po[512];
    if (orc_hungarian(n, q, p, P_in, P_out, Po, cost, Rt) == 0) bad += !is_perm(n, Po);
    free(p); free(adj); free(gains); free(fidx); free(q); free(vel); free(P_in); free(P_out);
    free(st); free(u); free(us); free(ca); free(who);
  }
  printf("sanitize driver: %s\n", bad ? "INVARIANT FAILURES" : "ok");
  return bad ? 1 : 0;
}
