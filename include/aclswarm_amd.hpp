/*
 * aclswarm_amd.hpp -- header-only C++ facade over the C ABI (aclswarm_amd.h)
 * with the reference's class and method names, for code written against
 * gitshitou/aclswarm's per-vehicle objects:
 *
 *   reference                                       facade (namespace acl::aclswarm::amd)
 *   ----------------------------------------------  -----------------------------------------
 *   Auctioneer        auctioneer.h:47-141           Auctioneer      -> acl_solve_batch (B = 1)
 *   DistCntrl         distcntrl.h:23-66             DistCntrl       -> acl_control_batch (B = 1)
 *   admm::Solver      lib/admm/include/admm/        admm::Solver    -> acl_admm_solve_batch (F = 1)
 *                     solver.h:16-60
 *
 * Layouts are the reference's (column-major Eigen storage): PtsMat n x 3 f64,
 * AdjMat n x n u8, GainMat 3n x 3n f64, AssignmentPerm indices() (vehicle ->
 * formation point, u8). Every method takes plain pointers in those layouts;
 * when <Eigen/Dense> is available the Eigen-typed overloads with the
 * reference's exact signatures are compiled too (ACLSWARM_AMD_HAVE_EIGEN).
 *
 * Semantics that differ from the reference, by design:
 *  - Auctioneer. In the reference every vehicle's object exchanges CBAA bids
 *    with its neighbours over ROS (setSendBidHandler -> network ->
 *    enqueueBid -> tick). Here the whole consensus runs on the GPU inside
 *    start(): the engine evaluates every vehicle's alignment and the rounds
 *    of lockstep-equivalent CBAA to the fixed point, and this object adopts
 *    the final table of ITS vehicle (vehid) exactly as
 *    auctioneer.cpp:250-295 does (isValidAssignment, shouldUseAssignment,
 *    the new-assignment handler, didConvergeOnInvalidAssignment). The
 *    result equals the reference's when all vehicles start from the same
 *    snapshot q (the synchronous case the parity tests pin). The send-bid
 *    handler is stored but never invoked, enqueueBid/tick accept and drop
 *    bids (no bids cross the network), and isIdle() is true whenever start()
 *    is not running.
 *  - Errors. The reference has none (asserts only); failures of the GPU
 *    layer (no device, out of memory, bad sizes) throw std::runtime_error
 *    with acl_last_error().
 *  - Each call is synchronous on the default HIP stream. For throughput use
 *    the batched C entry points (one call for B swarms); this facade is for
 *    drop-in use, one swarm at a time.
 *
 * Locking mirrors the reference (auctioneer.h:133-134): start() and tick()
 * serialize on the auction mutex and the new-assignment handler runs while
 * it is held (auctioneer.cpp:119,280); enqueueBid takes the queue mutex;
 * DistCntrl::compute does not lock.
 */
#ifndef ACLSWARM_AMD_HPP
#define ACLSWARM_AMD_HPP

#include <stddef.h>
#include <stdint.h>

#include <cmath>
#include <cstring>
#include <functional>
#include <iostream>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "aclswarm_amd.h"

#if defined(__has_include)
#if __has_include(<Eigen/Dense>)
#include <Eigen/Dense>
#define ACLSWARM_AMD_HAVE_EIGEN 1
#endif
#endif

namespace acl {
namespace aclswarm {
namespace amd {

using vehidx_t = uint8_t;  // utils.h:25

/* C callback of the new-assignment event: P (vehicle -> formation point). */
typedef void (*acl_new_assignment_fn)(void* user, const vehidx_t* P, int32_t n);

namespace detail {

inline void check(acl_status_t s) {
  if (s != ACL_OK) throw std::runtime_error(acl_last_error());
}

/* Owning device allocation (acl_malloc / acl_free). */
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  ~DeviceBuffer() { release(); }
  void* reserve(size_t bytes) {
    if (bytes > cap_) {
      release();
      check(acl_malloc(&p_, bytes));
      cap_ = bytes;
    }
    return p_;
  }
  void release() {
    if (p_) acl_free(p_);
    p_ = nullptr;
    cap_ = 0;
  }
  void* get() const { return p_; }
  template <class T> T* as() const { return static_cast<T*>(p_); }
  void upload(const void* src, size_t bytes) {
    reserve(bytes);
    check(acl_memcpy_h2d(p_, src, bytes, nullptr));
  }

 private:
  void* p_ = nullptr;
  size_t cap_ = 0;
};

/* One formation in the engine's device layout (aclswarm_amd.h "formation
 * table"): points [n][3], adjacency bit rows, 9 gain edge planes. */
struct DeviceFormation {
  int n = 0;
  int planes = 9;
  bool has_gains = false;
  DeviceBuffer p, adj, gains, off;

  void upload(int n_, const double* p_colmajor, const uint8_t* adj_colmajor,
              const double* gains_colmajor) {
    n = n_;
    const int W = (n + 63) / 64;
    std::vector<double> pr((size_t)3 * n);
    for (int i = 0; i < n; ++i)
      for (int c = 0; c < 3; ++c) pr[(size_t)3 * i + c] = p_colmajor[(size_t)c * n + i];
    std::vector<uint64_t> bits((size_t)n * W);
    check(acl_pack_adjacency(n, adj_colmajor, bits.data()));
    p.upload(pr.data(), pr.size() * 8);
    adj.upload(bits.data(), bits.size() * 8);
    int64_t zero = 0;
    off.upload(&zero, 8);
    has_gains = gains_colmajor != nullptr;
    if (has_gains) {
      // the 40-byte record stream when the blocks have the ADMM structure
      planes = acl_gain_planes(n, adj_colmajor, gains_colmajor);
      const int64_t E = acl_count_edges(n, adj_colmajor);
      std::vector<double> pl((size_t)(planes * (E > 0 ? E : 1)), 0.0);
      check(acl_pack_gains_planes(n, adj_colmajor, gains_colmajor, planes, pl.data()));
      gains.upload(pl.data(), pl.size() * 8);
    }
  }

  acl_formations_t table() const {
    acl_formations_t F;
    F.n = n;
    F.n_formations = 1;
    F.p = p.as<const double>();
    F.adj = adj.as<const uint64_t>();
    F.gains = has_gains ? gains.as<const double>() : nullptr;
    F.gain_off = off.as<const int64_t>();
    F.gain_planes = planes;
    F.gains_tiled = nullptr;
    return F;
  }
};

/* PtsMat (column-major n x 3) -> the engine's [n][3]. */
inline std::vector<double> rows_xyz(int n, const double* colmajor) {
  std::vector<double> r((size_t)3 * n);
  for (int i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c) r[(size_t)3 * i + c] = colmajor[(size_t)c * n + i];
  return r;
}

}  // namespace detail

// ============================================================================
// Auctioneer (auctioneer.h:47-141, auctioneer.cpp)
// ============================================================================

class Auctioneer {
 public:
  /* auctioneer.h:31-34 */
  struct Bid {
    std::vector<float> price;
    std::vector<int> who;
  };
  using BidConstPtr = std::shared_ptr<const Bid>;

  Auctioneer(vehidx_t vehid, uint8_t n, bool verbose = false)
      : n_(n), vehid_(vehid), verbose_(verbose) {
    if (n_ < 1 || vehid_ >= n_) throw std::runtime_error("Auctioneer: vehid >= n");
    P_.resize(n_);
    Pt_.resize(n_);
    for (int i = 0; i < n_; ++i) P_[i] = Pt_[i] = (vehidx_t)i;
  }

  void setNewAssignmentHandler(std::function<void(const std::vector<vehidx_t>&)> f) {
    handler_ = std::move(f);
  }
  /* C callback form: f(user, P, n). */
  void setNewAssignmentHandler(acl_new_assignment_fn f, void* user) {
    if (!f) { handler_ = nullptr; return; }
    handler_ = [f, user](const std::vector<vehidx_t>& P) { f(user, P.data(), (int32_t)P.size()); };
  }
  /* Stored, never invoked: bids do not leave the GPU (see file header). */
  void setSendBidHandler(std::function<void(uint32_t, uint32_t, const BidConstPtr&)> f) {
    send_bid_ = std::move(f);
  }

  /* auctioneer.cpp:42-61: new formation; assignment reset to identity and the
   * next auction's result is adopted unconditionally. p column-major n x 3,
   * adjmat column-major n x n. */
  void setFormation(const double* p_colmajor, const uint8_t* adj_colmajor) {
    form_.upload(n_, p_colmajor, adj_colmajor, nullptr);
    auction_open_ = false;
    formation_just_received_ = true;
    for (int i = 0; i < n_; ++i) P_[i] = Pt_[i] = (vehidx_t)i;
  }

  /* auctioneer.cpp:78-125 + 245-306: run the auction on snapshot q (column-
   * major n x 3) to consensus and adopt this vehicle's result. */
  void start(const double* q_colmajor) {
    std::lock_guard<std::mutex> lock(auction_mtx_);
    if (form_.n != n_) throw std::runtime_error("Auctioneer::start before setFormation");
    auction_open_ = true;
    auctionid_++;
    if (verbose_)  // auctioneer.cpp:110-115
      std::cout << std::endl << "********* Starting auction " << auctionid_ << " *********"
                << std::endl << std::endl;
    const int n = n_;
    const std::vector<double> q = detail::rows_xyz(n, q_colmajor);
    std::vector<uint16_t> Pin(n);
    for (int i = 0; i < n; ++i) Pin[i] = P_[i];
    const int32_t fidx = 0;
    d_q_.upload(q.data(), q.size() * 8);
    d_pin_.upload(Pin.data(), (size_t)n * 2);
    d_fidx_.upload(&fidx, 4);
    d_pout_.reserve((size_t)n * 2);
    d_status_.reserve(sizeof(acl_swarm_status_t));
    d_who_.reserve((size_t)n * n * 2);
    d_ws_.reserve(acl_solve_workspace_bytes(n, 1));

    const acl_formations_t F = form_.table();
    acl_solve_args_t a;
    std::memset(&a, 0, sizeof(a));
    a.B = 1;
    a.fidx = d_fidx_.as<const int32_t>();
    a.q = d_q_.as<const double>();
    a.P_in = d_pin_.as<const uint16_t>();
    a.P_out = d_pout_.as<uint16_t>();
    a.status = d_status_.as<acl_swarm_status_t>();
    a.who = d_who_.as<uint16_t>();
    a.workspace = d_ws_.get();
    acl_default_cntrl_gains(&a.cntrl);
    acl_default_safety_params(&a.safety);
    a.early_exit = 1;
    a.do_control = 0;
    detail::check(acl_solve_batch(&F, &a, nullptr));
    std::vector<uint16_t> who(n);  // this vehicle's final table: task -> vehicle
    detail::check(acl_memcpy_d2h(who.data(), d_who_.as<uint16_t>() + (size_t)vehid_ * n,
                                 (size_t)n * 2, nullptr));
    detail::check(acl_stream_synchronize(nullptr));
    finish(who);
    auction_open_ = false;
  }

  /* Accepted and dropped: the consensus ran inside start(). */
  void enqueueBid(vehidx_t, uint32_t, uint32_t, const Bid&) {
    std::lock_guard<std::mutex> lock(queue_mtx_);
  }
  void tick() { std::lock_guard<std::mutex> lock(auction_mtx_); }

  /* auctioneer.cpp:65-74 */
  void flush() {
    auction_open_ = false;
    invalid_assignment_ = false;
  }

  /* P: vehicle -> formation point; Pt: formation point -> vehicle. */
  std::vector<vehidx_t> getAssignment() const { return P_; }
  std::vector<vehidx_t> getInvAssignment() const { return Pt_; }
  void setAssignment(const vehidx_t* P) {
    for (int i = 0; i < n_; ++i) {
      P_[i] = P[i];
      Pt_[P[i]] = (vehidx_t)i;
    }
  }

  bool isIdle() const { return !auction_open_; }
  bool didConvergeOnInvalidAssignment() const { return invalid_assignment_; }
  int auctionId() const { return auctionid_; }

#ifdef ACLSWARM_AMD_HAVE_EIGEN
  using PtsMat = Eigen::Matrix<double, Eigen::Dynamic, 3>;
  using AdjMat = Eigen::Matrix<vehidx_t, Eigen::Dynamic, Eigen::Dynamic>;
  using AssignmentPerm = Eigen::PermutationMatrix<Eigen::Dynamic, Eigen::Dynamic, vehidx_t>;
  void setNewAssignmentHandler(std::function<void(const AssignmentPerm&)> f) {
    if (!f) { handler_ = nullptr; return; }
    handler_ = [f](const std::vector<vehidx_t>& P) {
      AssignmentPerm perm((int)P.size());
      for (size_t i = 0; i < P.size(); ++i) perm.indices()(i) = P[i];
      f(perm);
    };
  }
  void setFormation(const PtsMat& p, const AdjMat& adjmat) {
    setFormation(p.data(), adjmat.data());
  }
  void start(const PtsMat& q) { start(q.data()); }
  AssignmentPerm getAssignmentPerm() const { return toPerm(P_); }
  AssignmentPerm getInvAssignmentPerm() const { return toPerm(Pt_); }
  void setAssignment(const AssignmentPerm& P) { setAssignment(P.indices().data()); }

 private:
  static AssignmentPerm toPerm(const std::vector<vehidx_t>& v) {
    AssignmentPerm perm((int)v.size());
    for (size_t i = 0; i < v.size(); ++i) perm.indices()(i) = v[i];
    return perm;
  }
#endif

 private:
  /* auctioneer.cpp:250-295 (adoption) and 310-321 (shouldUseAssignment). */
  void finish(const std::vector<uint16_t>& who) {
    const int n = n_;
    std::vector<char> seen(n, 0);
    bool valid = true;
    for (int j = 0; j < n; ++j) {
      const unsigned v = who[j];
      if (v >= (unsigned)n || seen[v]) { valid = false; break; }
      seen[v] = 1;
    }
    if (!valid) {
      std::cout << "\033[95;1mInvalid Assignment\033[0m" << std::endl;
      invalid_assignment_ = true;
      return;
    }
    std::vector<vehidx_t> newPt(n), newP(n);
    for (int j = 0; j < n; ++j) {
      newPt[j] = (vehidx_t)who[j];
      newP[who[j]] = (vehidx_t)j;
    }
    bool use = true;
    if (formation_just_received_) formation_just_received_ = false;
    else if (newP == P_) use = false;
    if (!use) return;
    P_ = newP;
    Pt_ = newPt;
    if (handler_) handler_(P_);
  }

  int n_;
  vehidx_t vehid_;
  bool verbose_;
  std::vector<vehidx_t> P_, Pt_;
  int auctionid_ = 0;
  bool auction_open_ = false;
  bool invalid_assignment_ = false;
  bool formation_just_received_ = false;
  std::mutex queue_mtx_, auction_mtx_;
  std::function<void(const std::vector<vehidx_t>&)> handler_;
  std::function<void(uint32_t, uint32_t, const BidConstPtr&)> send_bid_;
  detail::DeviceFormation form_;
  detail::DeviceBuffer d_q_, d_pin_, d_fidx_, d_pout_, d_status_, d_who_, d_ws_;
};

// ============================================================================
// DistCntrl (distcntrl.h:23-66, distcntrl.cpp:20-102)
// ============================================================================

class DistCntrl {
 public:
  /* distcntrl.h:26-34, plain layouts: adjmat column-major n x n u8, gains
   * column-major 3n x 3n, qdes column-major n x 3; dstar_* column-major n x n
   * (filled by setFormation as the reference does). */
  struct Formation {
    std::string name;
    std::vector<uint8_t> adjmat;
    std::vector<double> gains;
    std::vector<double> qdes;
    std::vector<double> dstar_xy;
    std::vector<double> dstar_z;
  };

  /* distcntrl.h:36-45 */
  struct Gains {
    double K1_xy, K2_xy, K1_z, K2_z, e_xy_thr, e_z_thr, kp, kd;
  };

  DistCntrl(vehidx_t vehid, uint8_t n) : vehid_(vehid), n_(n) {
    if (n_ < 1 || vehid_ >= n_) throw std::runtime_error("DistCntrl: vehid >= n");
    acl_default_cntrl_gains(&g_);
    P_.resize(n_);
    for (int i = 0; i < n_; ++i) P_[i] = (vehidx_t)i;
  }

  void setGains(const Gains& g) {
    g_.K1_xy = g.K1_xy; g_.K2_xy = g.K2_xy; g_.K1_z = g.K1_z; g_.K2_z = g.K2_z;
    g_.e_xy_thr = g.e_xy_thr; g_.e_z_thr = g.e_z_thr; g_.kp = g.kp; g_.kd = g.kd;
  }

  /* distcntrl.cpp:28-35: keeps the shared formation, fills its dstar matrices
   * (utils::pdistmat, utils.h:137-147) and uploads it. */
  void setFormation(const std::shared_ptr<Formation>& f) {
    const int n = n_;
    if (!f || (int)f->qdes.size() != 3 * n || (int)f->adjmat.size() != n * n ||
        f->gains.size() != (size_t)9 * n * n)
      throw std::runtime_error("DistCntrl::setFormation: formation sizes do not match n");
    formation_ = f;
    pdist(f->qdes.data(), 0, 2, f->dstar_xy);
    pdist(f->qdes.data(), 2, 3, f->dstar_z);
    form_.upload(n, f->qdes.data(), f->adjmat.data(), f->gains.data());
  }

  /* distcntrl.cpp:38-41; P: vehicle -> formation point. */
  void setAssignment(const vehidx_t* P) {
    for (int i = 0; i < n_; ++i) P_[i] = P[i];
  }

  /* distcntrl.cpp:46-102: u for this vehicle from the snapshot q_veh
   * (column-major n x 3, vehicle space) and its velocity vel[3]. */
  void compute(const double* q_veh_colmajor, const double vel[3], double u[3]) {
    if (!formation_) throw std::runtime_error("DistCntrl::compute before setFormation");
    const int n = n_;
    const std::vector<double> q = detail::rows_xyz(n, q_veh_colmajor);
    std::vector<double> v((size_t)3 * n, 0.0);
    for (int c = 0; c < 3; ++c) v[(size_t)3 * vehid_ + c] = vel[c];
    std::vector<uint16_t> P(n);
    for (int i = 0; i < n; ++i) P[i] = P_[i];
    const int32_t fidx = 0;
    d_q_.upload(q.data(), q.size() * 8);
    d_vel_.upload(v.data(), v.size() * 8);
    d_p_.upload(P.data(), (size_t)n * 2);
    d_fidx_.upload(&fidx, 4);
    d_u_.reserve((size_t)3 * n * 8);
    d_status_.reserve(sizeof(acl_swarm_status_t));
    d_ws_.reserve(acl_solve_workspace_bytes(n, 1));
    const acl_formations_t F = form_.table();
    acl_control_args_t a;
    std::memset(&a, 0, sizeof(a));
    a.B = 1;
    a.fidx = d_fidx_.as<const int32_t>();
    a.q = d_q_.as<const double>();
    a.vel = d_vel_.as<const double>();
    a.P = d_p_.as<const uint16_t>();
    a.u = d_u_.as<double>();
    a.status = d_status_.as<acl_swarm_status_t>();
    a.workspace = d_ws_.get();
    a.cntrl = g_;
    acl_default_safety_params(&a.safety);
    detail::check(acl_control_batch(&F, &a, nullptr));
    detail::check(acl_memcpy_d2h(u, d_u_.as<double>() + (size_t)3 * vehid_, 24, nullptr));
    detail::check(acl_stream_synchronize(nullptr));
  }

#ifdef ACLSWARM_AMD_HAVE_EIGEN
  using PtsMat = Eigen::Matrix<double, Eigen::Dynamic, 3>;
  using AssignmentPerm = Eigen::PermutationMatrix<Eigen::Dynamic, Eigen::Dynamic, vehidx_t>;
  void setAssignment(const AssignmentPerm& P) { setAssignment(P.indices().data()); }
  Eigen::Vector3d compute(const PtsMat& q_veh, const Eigen::Vector3d vel) {
    Eigen::Vector3d u;
    compute(q_veh.data(), vel.data(), u.data());
    return u;
  }
#endif

 private:
  // squareform(pdist(M)) over columns [c0, c1) of the n x 3 matrix, by the
  // reference's |x|^2 + |y|^2 - 2 x'y identity (utils.h:140-146)
  void pdist(const double* M, int c0, int c1, std::vector<double>& D) const {
    const int n = n_;
    std::vector<double> N(n, 0.0);
    for (int i = 0; i < n; ++i)
      for (int c = c0; c < c1; ++c) N[i] += M[(size_t)c * n + i] * M[(size_t)c * n + i];
    D.assign((size_t)n * n, 0.0);
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) {
        double dot = 0.0;
        for (int c = c0; c < c1; ++c) dot += M[(size_t)c * n + i] * M[(size_t)c * n + j];
        D[(size_t)j * n + i] = std::sqrt(N[i] + N[j] - 2.0 * dot);
      }
  }

  vehidx_t vehid_;
  int n_;
  acl_cntrl_gains_t g_;
  std::vector<vehidx_t> P_;
  std::shared_ptr<Formation> formation_;
  detail::DeviceFormation form_;
  detail::DeviceBuffer d_q_, d_vel_, d_p_, d_fidx_, d_u_, d_status_, d_ws_;
};

// ============================================================================
// admm::Solver (lib/admm/include/admm/solver.h:16-60, solver.cpp:28-79)
// ============================================================================

namespace admm {

class Solver {
 public:
  /* solver.h:18-31, same names and defaults */
  struct Params {
    bool verbose = false;
    double thrSparseZero = 1e-8;
    double thrPlanar = 1e-2;
    double epsEig = 1e-5;
    double mu = 1;
    double thresh = 1e-4;
    double threshTr = 0.10;
    size_t maxItr = 10;
  };

  Solver() : Solver(Params()) {}
  explicit Solver(const Params& params) : params_(params) {}

  /* Gains for n points: pts column-major 3 x n, adj column-major n x n f64,
   * gains out column-major 3n x 3n. */
  void solve(int n, const double* pts_3xn, const double* adj_nxn, double* gains_out) {
    if (n < 1) throw std::runtime_error("admm::Solver::solve: n < 1");
    acl_admm_params_t p;
    acl_default_admm_params(&p);
    p.verbose = params_.verbose ? 1 : 0;
    p.thrSparseZero = params_.thrSparseZero;
    p.thrPlanar = params_.thrPlanar;
    p.epsEig = params_.epsEig;
    p.mu = params_.mu;
    p.thresh = params_.thresh;
    p.threshTr = params_.threshTr;
    p.maxItr = (int32_t)params_.maxItr;
    const size_t nn = (size_t)n * n;
    d_pts_.upload(pts_3xn, (size_t)3 * n * 8);
    d_adj_.upload(adj_nxn, nn * 8);
    d_gains_.reserve(9 * nn * 8);
    d_iters_.reserve(8);
    detail::check(acl_admm_solve_batch(1, n, d_pts_.as<const double>(), d_adj_.as<const double>(),
                                       d_gains_.as<double>(), d_iters_.as<int32_t>(), &p,
                                       nullptr));
    detail::check(acl_memcpy_d2h(gains_out, d_gains_.get(), 9 * nn * 8, nullptr));
    detail::check(acl_memcpy_d2h(iters_, d_iters_.get(), 8, nullptr));
    detail::check(acl_stream_synchronize(nullptr));
  }

  /* ADMM iteration counts of the last solve (2-D, 1-D); negative when the
   * PSD projection's sign iteration did not converge (aclswarm_amd.h). */
  int iterations2d() const { return iters_[0]; }
  int iterations1d() const { return iters_[1]; }

#ifdef ACLSWARM_AMD_HAVE_EIGEN
  Eigen::MatrixXd solve(const Eigen::Matrix<double, 3, Eigen::Dynamic>& pts,
                        const Eigen::MatrixXd& adj) {
    const int n = (int)pts.cols();
    Eigen::MatrixXd A(3 * n, 3 * n);
    solve(n, pts.data(), adj.data(), A.data());
    return A;
  }
#endif

 private:
  Params params_;
  int32_t iters_[2] = {0, 0};
  detail::DeviceBuffer d_pts_, d_adj_, d_gains_, d_iters_;
};

}  // namespace admm

}  // namespace amd
}  // namespace aclswarm
}  // namespace acl

#endif  // ACLSWARM_AMD_HPP
