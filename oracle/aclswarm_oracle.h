/*
 * aclswarm_oracle.h -- CPU restatement of aclswarm's hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the parity checker for the
 * MI355X engine (aclswarm_amd). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. The product never links it.
 *
 * What it restates (paths relative to the reference root):
 *   - Eigen 3.3.4 JacobiSVD on a 2x2 matrix and Eigen::umeyama (2-D, no
 *     scaling), as called by Auctioneer::alignFormation
 *     (aclswarm/src/auctioneer.cpp:347-415). Eigen is an unpinned third-party
 *     dependency ("3.2.2 or later", aclswarm/CMakeLists.txt:30-32) absent from
 *     the container; its published algorithm is restated in DESIGN.md §3.
 *   - CBAA: start/processBid/updateTaskAssignment/selectTaskAssignment/
 *     getPrice/isValidAssignment (auctioneer.cpp:78-120,182-306,325-343,
 *     469-549) in lockstep-equivalent rounds.
 *   - utils::pdistmat (aclswarm/include/aclswarm/utils.h:137-147) and
 *     DistCntrl::compute (aclswarm/src/distcntrl.cpp:46-102).
 *   - Safety::cmdinCb saturation and Safety::collisionAvoidance
 *     (aclswarm/src/safety.cpp:172-197, 412-541), utils::wrapToPi/closest
 *     (utils.h:275-325).
 *
 * Parity status. No reference test pins CBAA, DistCntrl or Safety (the only
 * C++ test is aclswarm/test/test_admm.cpp) and the reference C++ cannot be
 * built here (needs Eigen3 + ROS). The alignment is pinned against the
 * reference's own Python `arun` (aclswarm/src/aclswarm/assignment.py:15-53)
 * through committed golden vectors (tests/golden/arun_*.json); the auction,
 * control and safety restatements are otherwise "parity unpinned" against
 * reference outputs and are cross-checked by independent formulations in
 * tests/test_oracle.py.
 *
 * Layouts (oracle-internal, row-major):
 *   points  q, p, vel : [n][3] doubles
 *   adj               : [n][n] u8, adj[i*n+j] = adjmat(i,j)
 *   gains             : [3n][3n] doubles, g[r*3n+c] = GainMat(r,c)
 *   P                 : [n] u16, vehicle -> formation point
 */
#ifndef ACLSWARM_ORACLE_H
#define ACLSWARM_ORACLE_H

#include <stdint.h>

#include "../include/aclswarm_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_NONE (-1)

/* Eigen JacobiSVD<MatrixXd>(A, ComputeFullU|ComputeFullV) for 2x2 A.
 * A, U, V column-major. Returns 0 on success, -1 if A is not finite
 * (Eigen returns InvalidInput and leaves U,V,sv unset). */
int orc_jacobi_svd2(const double A[4], double U[4], double sv[2], double V[4]);

/* Eigen::umeyama(src, dst, false) for 2 x k point sets.
 * src/dst are [k][2] (point-major). R row-major 2x2, t[2].
 * variant 0 = Eigen 3.3.x rank rule, 1 = Eigen 3.4 det(U)det(V) rule. */
int orc_umeyama2(int k, const double* src, const double* dst, double R[4],
                 double t[2], int variant);

/* orc_umeyama2 (variant 0) plus the decision gap of its determinant-sign
 * and rank tests (the margin of include/aclswarm_amd.h); gap may be NULL. */
int orc_umeyama2_gap(int k, const double* src, const double* dst, double R[4],
                     double t[2], int variant, double* gap);

/* Auctioneer::alignFormation for vehicle v: R (row-major 2x2), t (2). */
/* The umeyama rule of every vehicle alignment below (orc_align*, the solve
 * entry points): 0 = Eigen 3.3.x (default), 1 = Eigen 3.4. Process-wide. */
void orc_set_umeyama_variant(int variant);
int orc_get_umeyama_variant(void);

void orc_align(int n, int v, const double* q, const double* p,
               const uint8_t* adj, const uint16_t* P, double R[4],
               double t[2]);

void orc_align_gap(int n, int v, const double* q, const double* p,
                   const uint8_t* adj, const uint16_t* P, double R[4],
                   double t[2], double* gap);

/* orc_prices plus the smallest alignment decision gap over the vehicles. */
void orc_prices_gap(int n, const double* q, const double* p, const uint8_t* adj,
                    const uint16_t* P, float* C, double* Rt, double* gap_min);

/* orc_prices_gap with each vehicle's own assignment: Prows (optional,
 * [n][n]) row v = vehicle v's assignment as formation point -> vehicle. */
void orc_prices_rows(int n, const double* q, const double* p, const uint8_t* adj,
                     const uint16_t* P, const uint16_t* Prows, float* C, double* Rt,
                     double* gap_min);

/* getPrice for every (vehicle v, task j) with v's own alignment:
 * C[v*n+j] = (float)(1.0 / (||q_v - (R_v p_j + t_v)|| + 1e-8)).
 * Rt (optional, [n][6]) receives R00,R01,R10,R11,t0,t1 per vehicle. */
void orc_prices(int n, const double* q, const double* p, const uint8_t* adj,
                const uint16_t* P, float* C, double* Rt);

/* Lockstep CBAA from the price matrix. who_out [n][n] int32 final tables
 * (vehicle rows, -1 = unassigned), price_out [n][n] float (may be NULL).
 * Returns eff_rounds = last round (1..2N) that changed any table, 0 if none.
 * early_exit=0 runs all 2N rounds literally. */
int orc_cbaa(int n, const float* C, const uint8_t* adj, const uint16_t* P,
             int early_exit, int32_t* who_out, float* price_out);

/* orc_cbaa plus the decision-margin tracker m[2] = (hi, lo) of the CBAA
 * comparisons (include/aclswarm_amd.h); m may be NULL. */
int orc_cbaa_m(int n, const float* C, const uint8_t* adj, const uint16_t* P,
               int early_exit, int32_t* who_out, float* price_out, float* m);
/* orc_cbaa_m with each vehicle's neighbours from its own assignment (Prows
 * as in orc_prices_rows; NULL: every vehicle uses P). */
int orc_cbaa_rows(int n, const float* C, const uint8_t* adj, const uint16_t* P,
                  const uint16_t* Prows, int early_exit, int32_t* who_out,
                  float* price_out, float* m);
void orc_margin_track(float* m, float hi, float lo);
double orc_margin_gap(const float* m);

/* utils::pdistmat on the xy columns and on the z column of p. */
void orc_pdist(int n, const double* p, double* dxy, double* dz);

/* DistCntrl::compute for vehicle v. Pt = the assignment's inverse
 * (formation point -> vehicle) this vehicle uses. */
void orc_control(int n, int v, const double* q, const double* vel_v,
                 const uint16_t* Pt, const uint8_t* adj, const double* gains,
                 const double* dxy, const double* dz,
                 const acl_cntrl_gains_t* g, double u[3]);

/* orc_control plus the gate margin: *gate_min = min(*gate_min, | |e| - thr |
 * / thr) over both gates of every edge (gate_min may be NULL). */
void orc_control_g(int n, int v, const double* q, const double* vel_v,
                   const uint16_t* Pt, const uint8_t* adj, const double* gains,
                   const double* dxy, const double* dz,
                   const acl_cntrl_gains_t* g, double u[3], double* gate_min);

/* Safety::cmdinCb saturation, in place on g[3]. */
void orc_saturate(const acl_safety_params_t* s, double g[3]);

/* Safety::collisionAvoidance for vehicle v, in place on g[3] (vx,vy,vz).
 * Returns VelocityGoal::modified. */
int orc_collision_avoidance(int n, int v, const double* q,
                            const acl_safety_params_t* s, double g[3]);

/* One full solve for one swarm (same contract as acl_solve_batch).
 * who_out [n][n] u16 (may be NULL); u, u_safe [n][3]; ca [n]. */
void orc_solve(int n, const double* q, const double* vel, const double* p,
               const uint8_t* adj, const double* gains, const uint16_t* P_in,
               const acl_cntrl_gains_t* g, const acl_safety_params_t* s,
               int early_exit, uint16_t* P_out, acl_swarm_status_t* st,
               double* u, double* u_safe, uint8_t* ca, uint16_t* who_out);

/* orc_solve plus the swarm's gate margin (acl_solve_args_t::gate_margin;
 * +inf without edges; may be NULL). */
void orc_solve_g(int n, const double* q, const double* vel, const double* p,
                 const uint8_t* adj, const double* gains, const uint16_t* P_in,
                 const acl_cntrl_gains_t* g, const acl_safety_params_t* s,
                 int early_exit, uint16_t* P_out, acl_swarm_status_t* st,
                 double* u, double* u_safe, uint8_t* ca, uint16_t* who_out,
                 double* gate_margin);

/* orc_solve_g for a swarm whose vehicles hold their own assignments
 * (acl_solve_args_t::P_rows): Prows [n][n], row v = vehicle v's assignment
 * as formation point -> vehicle, with Prows[v][P_in[v]] == v; each vehicle
 * aligns (auctioneer.cpp:357,369), finds its neighbours (:422-427) and, with
 * an invalid final table, keeps its assignment from its own row. A row that
 * is not such a permutation is BAD_INPUT. Prows NULL: orc_solve_g. */
void orc_solve_rows(int n, const double* q, const double* vel, const double* p,
                    const uint8_t* adj, const double* gains, const uint16_t* P_in,
                    const uint16_t* Prows, const acl_cntrl_gains_t* g,
                    const acl_safety_params_t* s, int early_exit, uint16_t* P_out,
                    acl_swarm_status_t* st, double* u, double* u_safe, uint8_t* ca,
                    uint16_t* who_out, double* gate_margin);

/* Batched solve over a thread pool (the CPU baseline). Swarm b uses
 * formation fidx[b]: p [F][n][3], adj [F][n][n], gains [F][3n][3n].
 * with_margin = 0 skips the decision-margin bookkeeping (not part of the
 * reference's work; status margin reported as 1). Returns wall seconds. */
double orc_solve_batch(int B, int n, int nthreads, const int32_t* fidx,
                       const double* q, const double* vel, const double* p,
                       const uint8_t* adj, const double* gains,
                       const uint16_t* P_in, const acl_cntrl_gains_t* g,
                       const acl_safety_params_t* s, int early_exit,
                       uint16_t* P_out, acl_swarm_status_t* st, double* u,
                       double* u_safe, uint8_t* ca, int with_margin);

/* ---- centralized comparator (hungarian_oracle.c) -------------------------
 * assignment.py:15-137 restated; see hungarian_oracle.c for the pinning. */
int orc_lsap(int n, const double* cost, int32_t* col4row);
void orc_arun2(int n, const double* qq, const double* p, double Rt[4]);
int orc_hungarian(int n, const double* q, const double* p,
                  const uint16_t* P_last, const uint16_t* P_cmp,
                  uint16_t* P_opt, double cost[2], double* Rt_out);

#ifdef __cplusplus
}
#endif

#endif
