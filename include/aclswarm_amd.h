/*
 * aclswarm_amd.h -- C ABI of the MI355X-native batched swarm-decision engine.
 *
 * This is the drop-in boundary for aclswarm's per-vehicle decision loop
 * (reference: gitshitou/aclswarm). Every entry point is plain C: device or
 * host pointers plus sizes, no C++/Eigen/torch types. Each declaration cites
 * the reference interface it replaces (paths relative to the reference root).
 *
 *   reference                                    this ABI
 *   -------------------------------------------  ----------------------------------
 *   Auctioneer::setFormation/start/.../          acl_solve_batch (auction part):
 *     processBid -> consensus -> P               B swarms x N vehicles in one call
 *     (aclswarm/src/auctioneer.cpp:42-306)
 *   DistCntrl::setFormation + compute            acl_solve_batch (control part)
 *     (aclswarm/src/distcntrl.cpp:28-102)
 *   Safety::cmdinCb saturation +                 acl_solve_batch (safety part)
 *     Safety::collisionAvoidance
 *     (aclswarm/src/safety.cpp:172-197,412-541)
 *   admm::Solver::solve                          acl_admm_solve_batch
 *     (aclswarm/lib/admm/src/solver.cpp:28-79)
 *   utils::pdistmat (aclswarm/include/aclswarm/utils.h:137-147)
 *                                                computed on device from p
 *
 * Layouts. The batched engine uses its own device layout, documented per
 * field below (row-major "xyz per vehicle" points, adjacency bitmasks, gain
 * blocks as 9 coalesced edge planes). acl_pack_* convert the reference's
 * column-major Eigen layouts (PtsMat n x 3, AdjMat n x n u8, GainMat 3n x 3n)
 * into it on the host.
 *
 * Index width. The reference uses uint8_t vehicle indices
 * (utils.h:25-30, vehidx_t), so N <= 255. The ABI widens indices to
 * uint16_t; for N <= 255 the semantics are identical ("who == -1" casts to
 * 0xFFFF here instead of 0xFF). acl_solve_batch accepts N <= 512 (config
 * C4 is N = 500): N <= 128 runs the LDS-resident auction kernel, larger N
 * the kernel whose CBAA `who` table lives in the workspace.
 *
 * Errors. The reference has no error channel (asserts compiled out in
 * Release, aclswarm/CMakeLists.txt:7-10); an invalid auction is a flag
 * (auctioneer.cpp:283-292). Here: argument errors return acl_status_t != 0,
 * per-swarm outcomes are flags in acl_swarm_status_t.
 *
 * Concurrency. acl_solve_batch is stream-ordered on the hipStream_t passed as
 * `void* stream` (NULL = default stream) and never synchronizes.
 * acl_admm_solve_batch synchronizes that stream between ADMM iterations (its
 * iteration control reads per-formation convergence flags back).
 */
#ifndef ACLSWARM_AMD_H
#define ACLSWARM_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACL_ABI_VERSION 11

typedef enum {
  ACL_OK = 0,
  ACL_ERR_INVALID_ARG = 1,
  ACL_ERR_UNSUPPORTED = 2, /* e.g. N above the kernel's supported maximum */
  ACL_ERR_HIP = 3,         /* a HIP runtime call failed */
  ACL_ERR_NO_DEVICE = 4
} acl_status_t;

/* DistCntrl::Gains (aclswarm/include/aclswarm/distcntrl.h:36-45). */
typedef struct {
  double K1_xy, K2_xy, K1_z, K2_z, e_xy_thr, e_z_thr, kp, kd;
} acl_cntrl_gains_t;

/* Safety parameters used by cmdinCb + collisionAvoidance
 * (aclswarm/src/safety.cpp:49-52). */
typedef struct {
  double max_vel_xy, max_vel_z, d_avoid_thresh, r_keep_out;
} acl_safety_params_t;

/* admm::Params (aclswarm/lib/admm/include/admm/solver.h:18-31), plus the
 * 2-D complement basis (not a reference parameter; ABI 6):
 *   ACL_ADMM_BASIS_LINPACK (default) -- the codegen's LINPACK dsvdc columns:
 *     gains identical to the reference's codegen ADMM (aclswarm/src/admm.cpp),
 *     including its violation of test_admm.cpp:84-187 on that formation;
 *   ACL_ADMM_BASIS_COMPLEX -- a complex-structured orthonormal basis of the
 *     same complement: the design is complex-linear and meets the graph rows,
 *     as aclswarm/test/test_admm.cpp:84-187 asserts of admm::Solver (the C++
 *     facade's admm::Solver uses it). Same kernel, same SDP, same loop. */
#define ACL_ADMM_BASIS_LINPACK 0
#define ACL_ADMM_BASIS_COMPLEX 1
typedef struct {
  int32_t verbose;
  double thrSparseZero;
  double thrPlanar;
  double epsEig;
  double mu;
  double thresh;
  double threshTr;
  int32_t maxItr;
  int32_t basis;   /* ACL_ADMM_BASIS_* */
} acl_admm_params_t;

/* Defaults: control gains from aclswarm/launch/coordination.launch:32-39,
 * safety from safety.cpp:49-52, ADMM from solver.h:18-31. */
void acl_default_cntrl_gains(acl_cntrl_gains_t* g);
void acl_default_safety_params(acl_safety_params_t* s);
void acl_default_admm_params(acl_admm_params_t* a);

/* ---- per-swarm outcome ------------------------------------------------- */
#define ACL_SWARM_VALID     0x01u /* every vehicle's final table is a permutation
                                     (isValidAssignment, auctioneer.cpp:325-343) */
#define ACL_SWARM_AGREE     0x02u /* all vehicles hold identical final tables */
#define ACL_SWARM_CHANGED   0x04u /* some vehicle adopted an assignment != P_in */
#define ACL_SWARM_NONFINITE 0x08u /* a bid price was NaN: exact ordered-scan path */
#define ACL_SWARM_BAD_INPUT 0x10u /* P_in not a permutation: swarm skipped */
#define ACL_SWARM_CA_ACTIVE 0x20u /* collision avoidance modified >= 1 command */
#define ACL_SWARM_FRAGILE   0x40u /* margin < ACL_FRAGILE_MARGIN: a last-ulp change
                                     of a compared value could change the outcome */
#define ACL_FRAGILE_MARGIN 1e-6

/* Decision margin (SURVEY §7 "Umeyama fidelity", §8b): the smallest relative
 * gap of the float comparisons that decided the swarm's outcome, over
 *   - every updateTaskAssignment evaluation (auctioneer.cpp:480-509) of
 *     vehicle v, task j: p1 = the winning price, p2 = the highest price in
 *     v's closed neighbourhood whose `who` differs from the winner's (a tie
 *     gives p2 = p1); gap (p1 - p2) / p1;
 *   - every selectTaskAssignment (auctioneer.cpp:521-541) of vehicle v,
 *     c_k = getPrice of task k, (price_k, who_k) its table entry, j* the
 *     selected task (if any), tasks with who_k == v skipped (a value compared
 *     with itself): j*: (c_j* - price_j*) / c_j*; another eligible task k:
 *     (c_j* - c_k) / c_j*; an ineligible task k with c_k > 0 that would be
 *     selected if it became eligible (no j*, c_k > c_j*, or c_k == c_j* and
 *     k < j*): (price_k - c_k) / price_k;
 *   - every alignment (Eigen::umeyama, auctioneer.cpp:397): the determinant
 *     sign test |det S| / (|S00 S11| + |S01 S10|) and the rank test
 *     |s1 - 1e-12 s0| / max(s1, 1e-12 s0) (0 when both are 0).
 * The f32 pairs are ranked exactly by their ratio p2/p1 (products of two
 * floats are exact in f64); the gap of the extreme pair is then computed in
 * f64 as (p1 - p2) / p1, or 1 when p2 < 2^-28 p1, and the swarm's margin is
 * the f64 minimum over all of it, rounded to f32 (1 when nothing was
 * compared, BAD_INPUT swarms included; 0 for NONFINITE swarms). Equal prices held by different vehicles
 * give margin 0. */

typedef struct {
  uint32_t flags;
  uint16_t eff_rounds; /* last CBAA round that changed any table (0..2N); the
                          state is a fixed point after it */
  uint16_t rounds;     /* the reference's round count, n * diameter = 2N
                          (auctioneer.cpp:50-51, 441-444) */
  uint16_t n_invalid;  /* vehicles whose final table is not a permutation */
  uint16_t n_ca;       /* vehicles whose command collision avoidance modified */
  float margin;        /* decision margin (above); in [0, 1] */
} acl_swarm_status_t; /* 16 bytes */

/* ---- formation table (device memory) ------------------------------------
 * Replaces DistCntrl::Formation (distcntrl.h:26-34) + Auctioneer::p_/adjmat_.
 * One table holds F formations of n vehicles; swarms index it by fidx.
 *   p        [F][n][3] f64   desired points (Formation::qdes), xyz per point
 *   adj      [F][n][W] u64   W = (n+63)/64; bit (j%64) of word (j/64) of row i
 *                            is adjmat(i,j). The auction uses the closed
 *                            neighbourhood (the diagonal does not matter).
 *   gains    f64 edge planes. Formation f has E_f directed edges (i,j) with
 *            adjmat(i,j) != 0, enumerated row-major (i, then j ascending);
 *            a diagonal entry is an edge of the control law too
 *            (distcntrl.cpp:62 does not skip j == i). Block A_ij = GainMat.block<3,3>(3i,3j)
 *            (distcntrl.cpp:66) is stored as 9 planes: element (r,c) of edge e
 *            at gains[9*gain_off[f] + (3r+c)*E_f + e].
 *   gain_off [F] i64         edge offset of formation f (prefix sum of E_f).
 *   gain_planes              9 (or 0): the layout above. 5: every block has
 *            the structure admm::Solver::solve assembles (solver.cpp:49-77:
 *            A = MatrixXd::Zero, the xy 2x2 block from the 2-D design, (2,2)
 *            from the 1-D design), i.e. exact +0.0 at (0,2), (1,2), (2,0),
 *            (2,1); only (0,0), (0,1), (1,0), (1,1), (2,2) are stored, as
 *            one 40-byte record per edge: entry k of edge e at
 *            gains[5*gain_off[f] + 5*e + k]. The control law still
 *            multiplies the structural zeros (0.0 * q in the same operation
 *            order), so both layouts give identical commands, NaN/Inf
 *            propagation included; the record stream is 40 B per edge
 *            instead of 72. acl_gain_planes tells which layout a GainMat
 *            admits.
 *   gains_tiled  optional (NULL = unused): the gain_planes == 5 records of
 *            every formation re-ordered by acl_tile_gains into 8 x 8 edge
 *            tiles (same per-formation offsets 5*gain_off[f]). Only
 *            acl_control_batch reads it (its pair kernel, n <= 128: every tile
 *            it processes is one contiguous run of records; same commands,
 *            bit for bit); acl_solve_batch's fused auction + control phase
 *            always reads the row-major `gains`. The two entry points'
 *            commands on the same assignment agree to about 1e-12 relative
 *            (the same terms summed in another order), not bit for bit.
 */
typedef struct {
  int32_t n;
  int32_t n_formations;
  const double* p;
  const uint64_t* adj;
  const double* gains;
  const int64_t* gain_off;
  int32_t gain_planes;
  const double* gains_tiled;
} acl_formations_t;

/* Zero-initialises *F (every optional pointer NULL, gain_planes 9) and sets
 * n and n_formations. ABI 3 added gains_tiled: a caller that fills the struct
 * field by field must start from this (or from a zeroed struct). */
void acl_formations_init(acl_formations_t* F, int32_t n, int32_t n_formations);

/* Formation-setup step (once per formation table, like acl_pack_gains; not
 * part of a solve): writes the tiled copy of F->gains (gain_planes must be 5,
 * n <= 128) to `out` (device, 5 * sum(E_f) doubles, not aliasing F->gains).
 * Tile order: tiles (I, J) with J >= I, row block by row block; a tile is
 * the 64 vertex pairs (8I + r, 8J + c), lane = 8r + c (on a diagonal tile
 * the lanes r <= c). Its records are two runs in lane order: edge (i, j) of
 * every lane that has one, then edge (j, i) of every lane that has one
 * (diagonal tile: lanes r < c). Stream-ordered. */
acl_status_t acl_tile_gains(const acl_formations_t* F, double* out, void* stream);

/* ---- swarm statistics of a solve ---------------------------
 * The convergence counters the multi-GPU gather all-reduces, computed from B
 * status records in one launch on `stream` (device pointers, no sync):
 *   counters[0 .. 10]  int64: B; the number of swarms with each of the
 *       flags VALID, AGREE, CHANGED, NONFINITE, BAD_INPUT, CA_ACTIVE,
 *       FRAGILE; the sums of n_invalid, n_ca and eff_rounds;
 *   counters[11 .. 74] int64: histogram of eff_rounds (bin 63: 63 or more);
 *   extrema[0..1]      f64: max eff_rounds, -(min margin) (0 and -1 for B = 0).
 * The reference keeps no such statistics in the hot path (its supervisor
 * logs convergence per trial, supervisor.py:297-348); the layout is the one
 * aclswarm_amd/dist.py reduces across ranks. */
#define ACL_STATS_COUNTERS 75
acl_status_t acl_swarm_stats(const acl_swarm_status_t* status, int32_t B, int64_t* counters,
                             double* extrema, void* stream);

/* ---- the batched solve --------------------------------------------------
 * One "solve" = for one swarm of n vehicles:
 *   (1) each vehicle's local 2-D Umeyama alignment of the formation to its
 *       neighbours (Auctioneer::alignFormation, auctioneer.cpp:347-415),
 *   (2) CBAA to consensus in lockstep-equivalent rounds
 *       (start/processBid/updateTaskAssignment/selectTaskAssignment,
 *       auctioneer.cpp:78-306,469-549), exact early exit at the fixed point,
 *   (3) adoption (isValidAssignment, auctioneer.cpp:250-295),
 *   (4) one DistCntrl::compute per vehicle with its adopted assignment
 *       (distcntrl.cpp:46-102),
 *   (5) Safety::cmdinCb saturation and Safety::collisionAvoidance
 *       (safety.cpp:172-197, 412-541).
 * All pointers are device pointers.
 *   fidx    [B]        formation of swarm b (0 <= fidx < F; a swarm with
 *                      fidx out of range gets BAD_INPUT like a bad P_in)
 *   q       [B][n][3]  vehicle positions, vehicle space (PtsMat q, one row
 *                      per vehicle)
 *   vel     [B][n][3]  vehicle velocities (the controller's damping input)
 *   P_in    [B][n]     assignment before the auction: vehicle -> formation
 *                      point (AssignmentPerm::indices())
 *   P_out   [B][n]     per-vehicle adopted formation point: the assignment
 *                      vehicle v adopts (its own table if valid, else P_in),
 *                      evaluated at v. Equals the consensus P when AGREE.
 *   status  [B]
 *   u       [B][n][3]  DistCntrl::compute (NULL to skip storing)
 *   u_safe  [B][n][3]  after saturation and collision avoidance (NULL ok)
 *   ca_flag [B][n]     VelocityGoal::modified (NULL ok)
 *   who     [B][n][n]  optional final CBAA tables, vehicle rows (NULL ok);
 *                      0xFFFF = unassigned (who == -1)
 *   workspace          device scratch of acl_solve_workspace_bytes(n, B)
 *                      bytes (required): the auction kernel hands each
 *                      vehicle's adopted assignment to the control kernels
 *                      through it; for n > 128 it also holds the CBAA tables.
 * The call enqueues three kernels on `stream` (n > 64: four, the alignment
 * first): the auction over all B swarms (with 5-entry gain records it also
 * runs DistCntrl, saturation and the collision test for every swarm whose
 * vehicles agree), the gain kernel (the other swarms) and the collision-
 * avoidance kernel for the vehicles they listed; and, unless ws_persistent,
 * a memset of the list counters before them.
 */
typedef struct {
  int32_t B;
  const int32_t* fidx;
  const double* q;
  const double* vel;
  const uint16_t* P_in;
  uint16_t* P_out;
  acl_swarm_status_t* status;
  double* u;
  double* u_safe;
  uint8_t* ca_flag;
  uint16_t* who;
  void* workspace;
  acl_cntrl_gains_t cntrl;
  acl_safety_params_t safety;
  int32_t early_exit; /* 1: stop at the first fixed point (bit-exact), 0: run
                         all 2N rounds like the reference */
  int32_t do_control; /* 0: auction only */
  double* align_Rt;   /* [B][n][6] optional (NULL ok): vehicle v's 2-D
                         alignment of the formation to its neighbourhood,
                         R row-major 2x2 then t (Auctioneer::alignFormation,
                         auctioneer.cpp:347-415); the `aligned` points of
                         logAssignment are R p + t (z unchanged) */
  double* gate_margin; /* [B] optional (NULL ok): the control law's gate
                          margin, min over the swarm's evaluated edges of
                          | |e| - thr | / thr for the gates |e_xy| > e_xy_thr
                          and |e_z| > e_z_thr (distcntrl.cpp:75,80); +inf
                          without edges. The gates themselves are decided on
                          correctly rounded e (the oracle's arithmetic) */
  int32_t skip_margin; /* ABI 7. 0 (default): status.margin is the decision
                          margin above. 1: the auction does not track it --
                          status.margin = -1, FRAGILE never set; assignments,
                          round counts and commands are the same bits (the
                          margin only observes the comparisons; n > 128 the
                          wide kernel's level walk stops at each winner). */
  const uint16_t* P_rows;   /* ABI 8. Optional (NULL: every swarm uses P_in)
                          [B][n][n]: for a swarm with P_rows_on[b] != 0, row v
                          is vehicle v's own assignment as formation point ->
                          vehicle (its Pt_), and P_in[b][v] must be v's point
                          in it (row v at P_in[b][v] holds v). Each vehicle
                          then aligns the formation with its own assignment
                          (auctioneer.cpp:357,369), takes its CBAA neighbours
                          from it (:422-427), and keeps it when its final
                          table is invalid -- the reference's auction while
                          the vehicles hold different assignments. A row that
                          is not such a permutation: BAD_INPUT. */
  const uint8_t* P_rows_on; /* [B] (with P_rows) */
  int32_t ws_persistent; /* ABI 10. 0 (default): the call zeroes the workspace's
                          collision-list counters first (one memset on the
                          stream). 1: the caller zero-filled the workspace
                          when it allocated it and has used it since only for
                          acl_solve_batch / acl_control_batch calls with the
                          same n and B (the counters' offset depends on both),
                          one stream at a time: every such call with control
                          leaves the counters zero (its collision-avoidance
                          launch resets them), so the call enqueues no memset
                          (a launch fewer per solve). */
} acl_solve_args_t;

/* Largest n acl_solve_batch accepts (512). */
int32_t acl_max_vehicles(void);

/* ACL_ABI_VERSION of the built library (a binding checks it at load time:
 * the status record and argument structs change between versions). */
int32_t acl_abi_version(void);

/* Bytes of device workspace acl_solve_batch needs for B swarms of n. */
size_t acl_solve_workspace_bytes(int32_t n, int32_t B);

acl_status_t acl_solve_batch(const acl_formations_t* formations,
                             const acl_solve_args_t* args, void* stream);

/* ---- host-side packing helpers (reference layouts -> device layout) ----- */
/* Number of directed edges (adjmat(i,j) != 0, diagonal included); adj is the
 * reference's column-major AdjMat (n x n u8). */
int64_t acl_count_edges(int32_t n, const uint8_t* adj_colmajor);
/* AdjMat (column-major n x n u8) -> [n][W] u64 bit rows. */
acl_status_t acl_pack_adjacency(int32_t n, const uint8_t* adj_colmajor,
                                uint64_t* out_bits);
/* GainMat (column-major 3n x 3n f64) -> 9 edge planes of E doubles
 * (E = acl_count_edges). */
acl_status_t acl_pack_gains(int32_t n, const uint8_t* adj_colmajor,
                            const double* gains_colmajor, double* out_planes);
/* 5 when every edge block of the GainMat has bit-exact +0.0 at (0,2), (1,2),
 * (2,0), (2,1) (ADMM-designed gains, solver.cpp:49-77), else 9. */
int32_t acl_gain_planes(int32_t n, const uint8_t* adj_colmajor, const double* gains_colmajor);
/* acl_pack_gains for either layout: planes = 9 as above, planes = 5 one
 * record (0,0), (0,1), (1,0), (1,1), (2,2) per edge, 5 E doubles (ACL_ERR if
 * a block breaks the structure). */
acl_status_t acl_pack_gains_planes(int32_t n, const uint8_t* adj_colmajor,
                                   const double* gains_colmajor, int32_t planes,
                                   double* out_planes);

/* ---- DistCntrl + Safety for given assignments (no auction) ---------------
 * DistCntrl::setAssignment + compute (distcntrl.cpp:38-102) and
 * Safety::cmdinCb/collisionAvoidance for B swarms whose assignment P is
 * already known (e.g. between auto-auctions, coordination_ros.cpp:370-378).
 * P [B][n] vehicle -> formation point; a P that is not a permutation (or a
 * fidx out of range) gives status BAD_INPUT and zero commands. status [B] gets flags (BAD_INPUT,
 * CA_ACTIVE) and n_ca; the other fields are zero. Device pointers; workspace
 * of acl_solve_workspace_bytes(n, B). Stream-ordered. */
typedef struct {
  int32_t B;
  const int32_t* fidx;
  const double* q;
  const double* vel;
  const uint16_t* P;
  double* u;
  double* u_safe;
  uint8_t* ca_flag;
  acl_swarm_status_t* status;
  void* workspace;
  acl_cntrl_gains_t cntrl;
  acl_safety_params_t safety;
  double* gate_margin; /* [B] optional, as in acl_solve_args_t */
} acl_control_args_t;

acl_status_t acl_control_batch(const acl_formations_t* formations,
                               const acl_control_args_t* args, void* stream);

/* ---- Auctioneer::logAssignment files (auctioneer.cpp:577-597) -----------
 * The reference's binary record, byte for byte (reader:
 * matlab/Helpers/read_alignment.m:1-19): u8 n, q f64[n*3] column-major,
 * adjmat u8[n*n] column-major, lastP u8[n], p f64[n*3] column-major,
 * aligned f64[n*3] column-major, P u8[n]. Host pointers; q and p are
 * [n][3] row-major here, adj is the column-major AdjMat, aligned is computed
 * from align_Rt exactly as alignFormation does (R p + t, z row identity).
 * n <= 255 (the format's u8 count). */
acl_status_t acl_write_assignment_log(const char* path, int32_t n, const double* q,
                                      const uint8_t* adj_colmajor, const uint16_t* lastP,
                                      const double* p, const double* align_Rt,
                                      const uint16_t* P);
/* Reads a record back: *n first (pass NULL buffers to query n), then the
 * arrays in the layouts acl_write_assignment_log takes (aligned [n][3]). */
acl_status_t acl_read_assignment_log(const char* path, int32_t* n, double* q,
                                     uint8_t* adj_colmajor, uint16_t* lastP, double* p,
                                     double* aligned, uint16_t* P);

/* ---- centralized Hungarian comparator -----------------
 * Replaces aclswarm/src/aclswarm/assignment.py:94-137
 * find_optimal_assignment(q, p, last), the reference's centralized baseline
 * for CBAA: align the formation to the whole swarm with 2-D Arun
 * (assignment.py:15-92, using the last assignment), cost S[v][j] =
 * ||q_v - paligned_j|| (scipy cdist), P = linear_sum_assignment(S)[1]
 * (SciPy's Crouse shortest-augmenting-path LSAP, tie-breaking included).
 * One wavefront per swarm; n <= 512. Device pointers:
 *   fidx    [B]        formation of swarm b (p of the formation table is used)
 *   q       [B][n][3]  vehicle positions
 *   P_last  [B][n]     last assignment, vehicle -> formation point (NULL =
 *                      identity, assignment.py:112-113)
 *   P_cmp   [B][n]     optional assignment to price under the same S (e.g.
 *                      acl_solve_batch's P_out): the optimality gap of CBAA
 *   P_opt   [B][n]     out: optimal vehicle -> formation point (0xFFFF on
 *                      BAD_INPUT / NONFINITE)
 *   cost    [B][2]     out: sum_v S[v][P_opt[v]], sum_v S[v][P_cmp[v]]
 *                      (NaN when P_cmp is NULL or not a permutation)
 *   align_Rt[B][4]     optional out {c, s, tx, ty}: paligned = (c px - s py
 *                      + tx, s px + c py + ty, pz)
 *   status  [B]        out: 0 or ACL_HUNG_* bits
 * Stream-ordered, no workspace. */
#define ACL_HUNG_BAD_INPUT   0x01 /* P_last not a permutation: swarm skipped */
#define ACL_HUNG_NONFINITE   0x02 /* a cost is NaN / -inf, or the matrix is
                                     infeasible (scipy raises ValueError) */
#define ACL_HUNG_CMP_INVALID 0x04 /* P_cmp given but not a permutation */

typedef struct {
  int32_t B;
  const int32_t* fidx;
  const double* q;
  const uint16_t* P_last;
  const uint16_t* P_cmp;
  uint16_t* P_opt;
  double* cost;
  double* align_Rt;
  int32_t* status;
} acl_hungarian_args_t;

acl_status_t acl_hungarian_batch(const acl_formations_t* formations,
                                 const acl_hungarian_args_t* args, void* stream);

/* ---- one vehicle's CBAA bid iteration, batched (ABI 11) -------------------
 * The message-level protocol of the per-vehicle Auctioneer, for vehicles
 * that exchange bids with their neighbours iteration by iteration
 * (Auctioneer::enqueueBid / tick / processBid, auctioneer.cpp:124-160,
 * 182-306) instead of running the whole consensus in acl_solve_batch: the
 * tally a vehicle runs once it holds all its neighbours' bids of an
 * iteration. For vehicle k of V (any swarms, one formation table):
 *   start[k] = 1  reset its table (price 0, who -1; auctioneer.cpp:448-465)
 *                 and make the START bid (selectTaskAssignment, :517-542);
 *   start[k] = 0  updateTaskAssignment (:469-513) over the candidates --
 *                 its own table and the neighbours' bids of the iteration,
 *                 the caller's std::map bids_curr_ after :475's insert of its
 *                 own bid, ascending vehid -- then selectTaskAssignment when
 *                 it was outbid.
 * Prices: getPrice(q_k, aligned_j) (:546-549) with aligned = (R p_j + t,
 * p_j.z) from the vehicle's alignment (acl_solve_batch's align_Rt row of
 * that vehicle, :400-414), evaluated on the device in the reference's f64
 * order: the same floats as acl_solve_batch's prices.
 * Device pointers:
 *   fidx       [V]        formation of vehicle k's swarm
 *   vehid      [V]        the vehicle's id in its swarm, < n
 *   q          [V][3]     its position (the auction's snapshot)
 *   Rt         [V][6]     its alignment {R00, R01, R10, R11, tx, ty}
 *   start      [V]        1: START bid, 0: a bid iteration
 *   price      [V][n]     in/out f32: its table's prices (Bid::price)
 *   who        [V][n]     in/out i32: its table's holders (Bid::who, -1 none)
 *   cand_off   [V + 1]    vehicle k's candidates are rows cand_off[k] ..
 *                         cand_off[k + 1] - 1 (>= 1 row unless start[k]),
 *                         0 <= cand_off[k] <= cand_off[k + 1] <= K
 *   cand_vehid [K]        each candidate's vehid, strictly ascending per vehicle
 *   cand_price [K][n] f32, cand_who [K][n] i32: the candidates' tables
 *                         (may be NULL when every start[k] is 1)
 *   task       [V]        out: the task the select took, -1 if none ran or
 *                         none was eligible
 *   flags      [V]        out: ACL_CBAA_* bits (BAD_INPUT: a vehid, fidx,
 *                         candidate range or candidate order is invalid; the
 *                         table is left as it was)
 * Stream-ordered, no workspace. */
#define ACL_CBAA_OUTBID    0x01 /* a task it held went to another vehicle */
#define ACL_CBAA_SELECTED  0x02 /* selectTaskAssignment took a task */
#define ACL_CBAA_BAD_INPUT 0x10

typedef struct {
  int32_t V;
  int32_t K;  /* rows of cand_vehid / cand_price / cand_who (cand_off[V] <= K) */
  const int32_t* fidx;
  const int32_t* vehid;
  const double* q;
  const double* Rt;
  const uint8_t* start;
  float* price;
  int32_t* who;
  const int32_t* cand_off;
  const int32_t* cand_vehid;
  const float* cand_price;
  const int32_t* cand_who;
  int32_t* task;
  int32_t* flags;
} acl_cbaa_step_args_t;

acl_status_t acl_cbaa_step_batch(const acl_formations_t* formations,
                                 const acl_cbaa_step_args_t* args, void* stream);

/* ---- closed-loop batched episodes ---------------------
 * B swarms flown for `steps` control periods in lockstep: the discrete-time
 * model of one vehicle's node graph (CoordinationROS + Safety) with a
 * perfectly tracking outer loop. Per control step k (global index
 * s = step0 + k):
 *   1. if s % auction_every == 0, the auto-auction
 *      (CoordinationROS::autoauctionCb, coordination_ros.cpp:322-359): a swarm
 *      whose previous auction converged on an invalid assignment flushes and
 *      skips this one (:339-345, Auctioneer::flush); otherwise CBAA from the
 *      current q (acl_solve_batch's auction from the vehicles' own
 *      assignments: P_in = P, and for a swarm flying per-vehicle tables each
 *      vehicle's own table as its P_rows row, so every vehicle aligns and
 *      finds its neighbours with its own assignment as in the reference),
 *      and each vehicle's adoption as auctioneer.cpp:250-295:
 *      an agreed valid result is adopted by every vehicle; an agreed invalid
 *      one sets `flush`; on disagreement each vehicle whose own final table
 *      is valid adopts it and the others keep theirs -- the swarm then flies
 *      per-vehicle tables (est.per_vehicle) until an agreed valid auction.
 *      A vehicle whose own table is invalid after a disagreeing auction keeps
 *      its old table and sets invalid_assignment_ (auctioneer.cpp:291): it
 *      flushes instead of starting the next auto-auction (:339-345), the
 *      others' auction stalls on its START bid (auctioneer.cpp:419-439) until
 *      the tick after, so `flush` is set and the swarm skips that auction
 *      (model limit: the stalled auction's stale START bids in the
 *      reference's queues, and a formation graph with several components,
 *      where only the flagged vehicle's component stalls, are not modelled);
 *   2. DistCntrl::compute with each vehicle's table and vel (controlCb,
 *      coordination_ros.cpp:365-378), Safety::cmdinCb saturation and collisionAvoidance
 *      (safety.cpp:172-197,412-541) -> the velocity goal;
 *   3. Safety::makeSafeTraj(control_dt, goal) (safety.cpp:330-408): rate
 *      limits on the goal velocity, room-bound clamps, goal position
 *      integration; the vehicle tracks the goal exactly (q <- goal.pos,
 *      vel <- goal.vel; the snap-stack outer loop and simulator are out of
 *      scope). Yaw is not carried: DIST goals have r = 0 (safety.cpp:181);
 *   4. if s % sample_every == 0, a supervisor tick (supervisor.py:297-337):
 *      |u| of every vehicle's DistCntrl command (voriggoal) and its
 *      collision_avoidance_active flag enter a ring of `bufflen` samples; once
 *      full, converged <=> every vehicle's window mean |u| <
 *      orig_zero_vel_thr, gridlocked <=> some vehicle's window mean CA flag >
 *      avg_active_ca_thr (means: sequential sum oldest -> newest, / bufflen).
 * Device pointers, updated in place so an episode can continue in chunks:
 *   fidx [B]; q, vel [B][n][3]; P [B][n] (vehicle -> its formation point:
 *   a permutation at the start; while a swarm flies per-vehicle tables,
 *   each vehicle's point in its own table); flush [B] u8;
 *   est [B] acl_episode_status_t; ring_u [B][bufflen][n] f64 and
 *   ring_ca [B][bufflen][n] u8 (zeroed with est before step 0; in est,
 *   converged_step and gridlock_step then set to -1).
 * Optional histories (NULL = not stored), k = local step:
 *   q_hist, vel_hist [steps][B][n][3] (state after step k), u_hist [steps][B][n][3]
 *   (DistCntrl output), ca_hist [steps][B][n], P_hist [steps][B][n]
 *   (each vehicle's point in the table used by step k's controller).
 * workspace: acl_episode_workspace_bytes(n, B) bytes. A continuing call
 * must get the same workspace when an auction is pending or a swarm flies
 * per-vehicle tables (both live there; est says which). */
typedef struct {
  double control_dt;       /* 0.01 s (coordination.launch:25, safety.cpp:38) */
  int32_t auction_every;   /* autoauction_dt / control_dt = 1.2 / 0.01 = 120
                              (coordination.launch:6,24) */
  int32_t sample_every;    /* control steps per supervisor tick: 100 Hz / 50 Hz
                              = 2 (supervisor.py:121) */
  int32_t bufflen;         /* BUFFER_SECONDS * tick_rate = 50 (supervisor.py:
                              47,126) */
  int32_t auction_latency; /* control steps from an auto-auction's start to the
                              adoption of its result. 0: within its own step
                              (instantaneous). > 0: that many steps. -1: the
                              reference's timing per swarm: the auctioneer
                              processes one bid per auctioneer_dt = 1 ms tick
                              (coordination.launch:23, auctioneer.cpp:139-160)
                              and a vehicle needs every neighbour's bid in each
                              of the 2n rounds (auctioneer.cpp:198-241), so
                              ceil(2 n d_max 1 ms / control_dt) steps, d_max
                              the formation graph's largest degree. Control
                              keeps the old assignment meanwhile; an auto-
                              auction that finds one pending restarts it
                              (coordination_ros.cpp:355-358: "Auctioneer is
                              busy! Restarting."). */
  double max_accel_xy;     /* 0.5 (safety.cpp:45) */
  double max_accel_z;      /* 0.8 (safety.cpp:46) */
  double bounds_min[3];    /* room bounds: trial.sh:96 {-100, -100, 0} */
  double bounds_max[3];    /*              {100, 100, 30} */
  double orig_zero_vel_thr;  /* 1.00 m/s (supervisor.py:61) */
  double avg_active_ca_thr;  /* 0.95 (supervisor.py:62) */
  int32_t assignment;      /* ABI 9. ACL_ASSIGN_CBAA (0, default): the auction
                              above. ACL_ASSIGN_CENTRAL: the reference's
                              centralized comparison mode
                              (/operator/central_assignment,
                              coordination_ros.cpp:330-343): at each
                              auto-auction the operator's
                              find_optimal_assignment(q, p, last)
                              (operator.py:219-240, assignment.py:94-137,
                              acl_hungarian_batch with P_last = the swarm's
                              current P) is applied as every vehicle's
                              setAssignment + newAssignmentCb -- no CBAA, no
                              flush rule, no auction latency; a swarm whose
                              Hungarian problem is BAD_INPUT / NONFINITE (the
                              operator's scipy call would raise) keeps its P
                              and counts n_invalid. n_auctions counts the
                              central assignments applied. */
} acl_episode_params_t;

#define ACL_ASSIGN_CBAA    0
#define ACL_ASSIGN_CENTRAL 1

void acl_default_episode_params(acl_episode_params_t* e);

typedef struct {
  int32_t converged_step;  /* first global step whose tick found has_converged, -1 */
  int32_t gridlock_step;   /* first global step whose tick found has_gridlocked, -1 */
  int32_t converged;       /* has_converged at the last tick */
  int32_t gridlocked;      /* has_gridlocked at the last tick */
  uint16_t n_auctions;     /* auctions run */
  uint16_t n_invalid;      /* auctions that converged on an invalid assignment */
  uint16_t n_skipped;      /* auctions skipped by the flush rule */
  uint16_t n_disagree;     /* auctions whose vehicles ended on different
                              tables (each adopted its own valid one) */
  uint32_t n_samples;      /* supervisor ticks taken */
  uint32_t n_ca_steps;     /* vehicle-steps with collision avoidance active */
  int32_t pending_step;    /* 1 + the global step at which the pending
                              auction's result is adopted, 0 if none
                              (auction_latency != 0; its result stays in the
                              workspace between calls): a zeroed status is the
                              start of an episode */
  uint16_t n_restarted;    /* auctions restarted before they completed */
  uint16_t per_vehicle;    /* 1: the swarm's vehicles fly different tables
                              (kept in the workspace) since a disagreeing
                              auction; 0 after an agreed valid one */
} acl_episode_status_t; /* 40 bytes */

typedef struct {
  int32_t B;
  const int32_t* fidx;
  double* q;
  double* vel;
  uint16_t* P;
  uint8_t* flush;
  acl_episode_status_t* est;
  double* ring_u;
  uint8_t* ring_ca;
  int32_t step0;
  int32_t steps;
  double* q_hist;
  double* vel_hist;
  double* u_hist;
  uint8_t* ca_hist;
  uint16_t* P_hist;
  void* workspace;
  acl_cntrl_gains_t cntrl;
  acl_safety_params_t safety;
  acl_episode_params_t ep;
} acl_episode_args_t;

size_t acl_episode_workspace_bytes(int32_t n, int32_t B);
acl_status_t acl_episode_batch(const acl_formations_t* formations,
                               const acl_episode_args_t* args, void* stream);

/* ---- batched Monte-Carlo trials (ABI 9; SURVEY §8f widening of row f1) ---
 * B independent trials of aclswarm_sim's supervisor (aclswarm_sim/nodes/
 * supervisor.py:160-236) over the closed loop of acl_episode_batch: each
 * swarm flies a sequence of K formations (its formation group, fseq[b][k])
 * through the supervisor's state machine
 *   HOVERING --HOVER_WAIT--> next_formation --> WAITING_ON_ASSIGNMENT
 *   --assignment--> FLYING (logging) --converged--> IN_FORMATION
 *   --CONVERGED_WAIT--> HOVERING ... --all K done--> COMPLETE
 *   FLYING --gridlocked--> GRIDLOCK --has_left_gridlock--> FLYING
 *   with the ASSIGNMENT (20 s), GRIDLOCK (90 s) and trial watchdog (600 s)
 *   timeouts --> TERMINATE,
 * its windowed predicates over their own sample buffers (a predicate appends
 * a sample only when the state machine calls it; next_state clears both
 * buffers except FLYING -> IN_FORMATION, supervisor.py:238-265,297-337), and
 * its per-trial record (the CSV row of complete(), :404-415): the smoothed
 * planar distance flown per vehicle (log_signals, :452-487), the time to
 * converge per formation, the (last) gridlock duration per formation and the
 * assignments received per formation.
 * Per control step s (control_dt), per swarm not yet COMPLETE / TERMINATE:
 *   1. a formation requested by the last supervisor tick is committed
 *      (CoordinationROS::spin, coordination_ros.cpp:95-153): the vehicles'
 *      controllers stop and send one zero command (makeSafeTraj of a zero
 *      velocity goal), the assignment resets to identity (Auctioneer::
 *      setFormation, auctioneer.cpp:42-62), flush clears, and the first
 *      auto-auction is due form_settle_time later, then one every
 *      auction_every steps (autoauctionCb, :322-359);
 *   2. a due auto-auction: CBAA with the episode's adoption and flush rules
 *      (acl_episode_batch step 1, auction_latency must be 0), or the
 *      operator's Hungarian (ep.assignment = ACL_ASSIGN_CENTRAL); a vehicle
 *      that adopts an assignment starts its controller (first_assignment_,
 *      newAssignmentCb :284-303); vehicle 0's assignment message is the
 *      supervisor's (assignmentCb, supervisor.py:147-150; in the centralized
 *      mode a message only when the assignment changed or is the first,
 *      centralAssignmentCb :271-280);
 *   3. DistCntrl + Safety for every vehicle whose controller runs, and
 *      makeSafeTraj of its safe command; a vehicle whose controller is
 *      stopped holds its last goal (Safety::controlCb keeps sending the last
 *      goal message, safety.cpp:268-290; perfectly tracked);
 *   4. every sample_every steps, one supervisor tick (tick_rate Hz): its
 *      voriggoal / CA samples are |u| and the CA flag of running
 *      controllers, 0 for stopped ones.
 * Model limits: the trial starts in HOVERING with the swarm in
 * the air (IDLE / TAKING_OFF are the simulator's); a formation commits at the
 * step after the tick that requested it (the 5 Hz spin loop's delay is not
 * modelled); the zero command's collision-avoidance flag is taken as 0; the
 * watchdog counts from the first tick.
 * Device pointers, updated in place (a trial continues across calls):
 *   fseq [B][K] formation indices (a trial with an index outside [0,
 *   n_formations) ends at once: TERMINATE, nothing of the table read, its
 *   fidx 0); fidx [B] out: the formation of each
 *   swarm's controllers; q, vel [B][n][3]; P [B][n] (identity at the start);
 *   flush [B]; ts [B] acl_trial_status_t (zeroed before the first call, then
 *   acl_trial_init); ctl_on [B][n] u8; ring_u [B][bufflen][n] f64,
 *   ring_ca [B][bufflen][n] u8 (the converged / gridlocked sample buffers);
 *   posf [B][2][n] f64 (the smoothed x / y of log_signals); dist [B][n];
 *   t_conv, t_avoid [B][K] f64 s; n_assign [B][K] i32.
 * Optional histories (NULL = not stored), k = local step: q_hist, vel_hist,
 *   u_hist [steps][B][n][3]; ca_hist, ctl_hist [steps][B][n] u8; P_hist
 *   [steps][B][n]; state_hist [steps][B] i32 (supervisor state after the
 *   step). workspace: acl_trial_workspace_bytes(n, B). */
enum {
  ACL_TRIAL_HOVERING = 3,             /* supervisor.py State values */
  ACL_TRIAL_WAITING_ON_ASSIGNMENT = 4,
  ACL_TRIAL_FLYING = 5,
  ACL_TRIAL_IN_FORMATION = 6,
  ACL_TRIAL_GRIDLOCK = 7,
  ACL_TRIAL_COMPLETE = 8,
  ACL_TRIAL_TERMINATE = 9
};

typedef struct {
  acl_episode_params_t ep;        /* control_dt, auction_every, sample_every
                                     (control steps per tick), bufflen
                                     (BUFFLEN), accelerations, bounds, the two
                                     thresholds, assignment; auction_latency
                                     must be 0 */
  int32_t tick_rate;              /* 50 Hz (supervisor.py:121) */
  int32_t settle_steps;           /* form_settle_time / control_dt = 150
                                     (coordination.launch:5) */
  double hover_wait;              /* 5 s (supervisor.py:52) */
  double assignment_timeout;      /* 20 s (:53) */
  double formation_received_wait; /* 1 s (:54) */
  double converged_wait;          /* 1 s (:55) */
  double gridlock_timeout;        /* 90 s (:56) */
  double trial_timeout;           /* 600 s (:57) */
  double alpha;                   /* 0.98 (:88, log_signals' smoothing) */
} acl_trial_params_t;

void acl_default_trial_params(acl_trial_params_t* t);

typedef struct {
  int32_t state;          /* ACL_TRIAL_* */
  int32_t last_state;
  int32_t timer_ticks;    /* supervisor timer (-1 on entering a state) */
  int32_t formation;      /* curr_formation_idx (-1 before the first) */
  int32_t ticks;          /* supervisor ticks since the trial started */
  int32_t received;       /* received_assignment */
  int32_t logging;        /* is_logging */
  int32_t commit;         /* 1: a formation waits to be committed */
  int32_t next_auction;   /* steps to the next auto-auction (0: none) */
  int32_t conv_len, conv_head;  /* 'converged_orig_vel' deque: size, next slot */
  int32_t grid_len, grid_head;  /* 'gridlocked_active_ca' deque */
  int32_t log_init;       /* log_signals' filters initialised */
  int32_t t_start;        /* step at which the formation's logging started */
  int32_t t_grid;         /* step at which GRIDLOCK was entered */
  int32_t done_step;      /* step of complete() / terminate(), -1 running */
  uint16_t n_auctions, n_invalid, n_skipped, n_disagree;
  int32_t per_vehicle;    /* the swarm's vehicles fly different tables */
} acl_trial_status_t; /* 80 bytes */

typedef struct {
  int32_t B;
  int32_t K;
  const int32_t* fseq;
  int32_t* fidx;
  double* q;
  double* vel;
  uint16_t* P;
  uint8_t* flush;
  acl_trial_status_t* ts;
  uint8_t* ctl_on;
  double* ring_u;
  uint8_t* ring_ca;
  double* posf;
  double* dist;
  double* t_conv;
  double* t_avoid;
  int32_t* n_assign;
  int32_t step0;
  int32_t steps;
  double* q_hist;
  double* vel_hist;
  double* u_hist;
  uint8_t* ca_hist;
  uint8_t* ctl_hist;
  uint16_t* P_hist;
  int32_t* state_hist;
  void* workspace;
  acl_cntrl_gains_t cntrl;
  acl_safety_params_t safety;
  acl_trial_params_t tp;
} acl_trial_args_t;

size_t acl_trial_workspace_bytes(int32_t n, int32_t B);
/* the start of a trial: ts zeroed except state HOVERING, timer_ticks -1,
   formation -1, done_step -1; P identity; ctl_on, rings, posf, dist, t_conv,
   t_avoid, n_assign, flush zeroed; fidx = fseq[b][0] (device pointers of
   acl_trial_args_t; q and vel are the caller's) */
acl_status_t acl_trial_init(const acl_trial_args_t* args, int32_t n, void* stream);
acl_status_t acl_trial_batch(const acl_formations_t* formations,
                             const acl_trial_args_t* args, void* stream);

/* ---- random formation groups on the device -----------
 * Replaces aclswarm_sim/nodes/generate_random_formation.py:59-80
 * generate_formation_group(n, fc, l, w, h, min_dist) after
 * np.random.seed(seeds[g]) (trial.sh:60): numpy's legacy MT19937 stream,
 * reproduced output for output, so the C2-C5 inputs are the reference
 * generator's own formations without a host round trip. One wavefront per
 * group. Device pointers:
 *   seeds   [F] u32
 *   points  [F][2][n][3] f64  formations 'A' and 'B', xyz per point
 *   adj     [F][n][n] u8      adjmat (ones - eye, minus the random pairs
 *                             unless fc)
 *   status  [F]               0, or bit k set: formation k needed more than
 *                             max_candidates samples (the reference gives up
 *                             after 5 s of wall clock, :35-53, and returns {})
 *   drawn   [F] i64           32-bit outputs consumed (NULL ok)
 * n in [1, 512]; a noncomplete group needs n >= 5 (randint(1, n - 3)). */
acl_status_t acl_generate_formation_groups(int32_t F, int32_t n, const uint32_t* seeds,
                                           int32_t fc, double l, double w, double h,
                                           double min_dist, int64_t max_candidates,
                                           double* points, uint8_t* adj, int32_t* status,
                                           int64_t* drawn, void* stream);

/* ---- ADMM formation-gain design (admm::Solver::solve, solver.cpp:28-79) -
 * F formations of n points: pts [F][3][n] column-major 3 x n per formation
 * (Eigen::Matrix<double,3,Dynamic>), adj [F][n][n] f64 (symmetric 0/1),
 * gains out [F][3n][3n] column-major. Device pointers. iters [F][2]
 * (2-D and 1-D ADMM iteration counts, may be NULL). The PSD projection of
 * each ADMM iteration (eigenvalues > epsEig kept, solver.cpp:296-316) is a
 * Newton-Schulz matrix-sign iteration on the matrix cores; a part whose sign
 * iteration does not converge in 64 steps (an eigenvalue within ~1e-11 |W|
 * of epsEig) is projected by a Jacobi eigendecomposition instead; if that
 * too is left unconverged after 40 sweeps the part's iters entry is the
 * negated count (-iterations): its gains are not reliable. params->basis
 * selects the 2-D complement basis (ACL_ADMM_BASIS_*; LINPACK by default). */
acl_status_t acl_admm_solve_batch(int32_t F, int32_t n, const double* pts,
                                  const double* adj, double* gains,
                                  int32_t* iters,
                                  const acl_admm_params_t* params,
                                  void* stream);

/* ---- minimal device-memory helpers (for callers without a framework) ---- */
int32_t acl_device_count(void);
acl_status_t acl_set_device(int32_t device);
acl_status_t acl_malloc(void** ptr, size_t bytes);
acl_status_t acl_free(void* ptr);
acl_status_t acl_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
acl_status_t acl_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
acl_status_t acl_memset(void* dst, int value, size_t bytes, void* stream);
acl_status_t acl_stream_synchronize(void* stream);
const char* acl_last_error(void);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* ACLSWARM_AMD_H */
