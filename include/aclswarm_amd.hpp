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
 * Types are the reference's (utils.h:25-30): vehidx_t, GainMat, AdjMat,
 * PtsMat, AssignmentVec, AssignmentPerm, and the methods carry the
 * reference's exact signatures (getAssignment() returns an AssignmentPerm
 * whose indices()(v) is vehicle v's formation point, DistCntrl::Formation
 * holds AdjMat / GainMat / PtsMat / MatrixXd, compute returns a Vector3d).
 * With <Eigen/Dense> they ARE the Eigen types (ACLSWARM_AMD_HAVE_EIGEN);
 * without it a small in-tree column-major matrix and permutation
 * (namespace mini below) provide the calls the reference's caller makes on
 * them: .indices()(v), .transpose(), .data(), (i, j), .cast<T>(), .rows(),
 * .cols(), .size(), isApprox, Map<const AssignmentVec>(ptr, n). Plain-pointer
 * forms in the column-major layouts stay available under *ColMajor names.
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
 *    handler is called once per auction, after the consensus, with this
 *    vehicle's final bid (the table the reference's vehicle holds after its
 *    last round: who, and each task's price rebuilt from the holder's
 *    alignment as getPrice computes it, auctioneer.cpp:546-549) and
 *    iter = 2n (cbaa_max_iter_), so a ROS-side wrapper can still publish a
 *    CBAA.msg per auction (coordination_ros.cpp:308-318); the per-round bids
 *    never leave the GPU. enqueueBid/tick accept and drop bids, and isIdle()
 *    is true whenever start() is not running.
 *    Exchange mode (setBidExchange(true), ABI 11) is the reference's message
 *    protocol instead, for fleets that mix these objects with other
 *    vehicles' Auctioneers: start() aligns on the GPU (acl_solve_batch, this
 *    vehicle's align_Rt row), makes the START bid and sends it (iter 0);
 *    enqueueBid queues neighbours' bids, tick() processes one as processBid
 *    does (auctioneer.cpp:182-306: iteration buckets, the START-bid bucket,
 *    bidIterComplete over the neighbours of this vehicle's own assignment),
 *    and each completed iteration's tally -- updateTaskAssignment and, when
 *    outbid, selectTaskAssignment -- runs on the GPU (acl_cbaa_step_batch,
 *    V = 1); after 2n iterations the vehicle adopts its table as above. With
 *    every vehicle starting from one snapshot the outcome equals the
 *    one-call consensus bit for bit (tests/test_gpu_facade.py).
 *  - Errors. The reference has none (asserts only). Auctioneer::start keeps
 *    that shape: a call it cannot run (no formation, q not n x 3, a GPU-layer
 *    failure) runs no auction, calls no handler and leaves the assignment as
 *    it was; lastStatus() returns the acl_status_t (ACL_OK after a good
 *    auction) and lastError() the message. The other facade calls
 *    throw std::runtime_error with acl_last_error() on GPU-layer failures
 *    (no device, out of memory, bad sizes).
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
#include <algorithm>
#include <atomic>
#include <iostream>
#include <map>
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

#ifndef ACLSWARM_AMD_HAVE_EIGEN
// ----------------------------------------------------------------------------
// Minimal stand-ins for the Eigen types of utils.h:25-30 when Eigen is absent:
// column-major dense storage and a permutation with Eigen's conventions
// (indices()(v) = the image of v; transpose() = the inverse).
// ----------------------------------------------------------------------------
namespace mini {

template <class T>
class Matrix {
 public:
  Matrix() = default;
  Matrix(int rows, int cols) : r_(rows), c_(cols), d_((size_t)rows * cols, T()) {}
  int rows() const { return r_; }
  int cols() const { return c_; }
  int size() const { return r_ * c_; }
  T* data() { return d_.data(); }
  const T* data() const { return d_.data(); }
  T& operator()(int i, int j) { return d_[(size_t)j * r_ + i]; }
  const T& operator()(int i, int j) const { return d_[(size_t)j * r_ + i]; }
  T& operator()(int i) { return d_[(size_t)i]; }  // vectors (and linear index)
  const T& operator()(int i) const { return d_[(size_t)i]; }
  void resize(int rows, int cols) {
    r_ = rows;
    c_ = cols;
    d_.assign((size_t)rows * cols, T());
  }
  void setZero() { std::fill(d_.begin(), d_.end(), T()); }
  Matrix transpose() const {
    Matrix t(c_, r_);
    for (int j = 0; j < c_; ++j)
      for (int i = 0; i < r_; ++i) t(j, i) = (*this)(i, j);
    return t;
  }
  template <class U>
  Matrix<U> cast() const {
    Matrix<U> m(r_, c_);
    for (int k = 0; k < size(); ++k) m.data()[k] = static_cast<U>(d_[(size_t)k]);
    return m;
  }
  // exact equality stands in for Eigen's fuzzy compare (index vectors)
  bool isApprox(const Matrix& o) const { return r_ == o.r_ && c_ == o.c_ && d_ == o.d_; }
  bool operator==(const Matrix& o) const { return isApprox(o); }
  static Matrix Zero(int rows, int cols) { return Matrix(rows, cols); }

 private:
  int r_ = 0, c_ = 0;
  std::vector<T> d_;
};

// Eigen::Map<const AssignmentVec>(ptr, n): a read-only view copied on use
template <class M>
class Map;
template <class T>
class Map<const Matrix<T>> {
 public:
  Map(const T* p, size_t n) : p_(p), n_((int)n) {}
  const T* data() const { return p_; }
  int size() const { return n_; }

 private:
  const T* p_;
  int n_;
};

class PermutationMatrix {
 public:
  using IndicesType = Matrix<vehidx_t>;
  PermutationMatrix() = default;
  explicit PermutationMatrix(int n) { setIdentity(n); }
  explicit PermutationMatrix(const IndicesType& idx) : idx_(idx) {}
  explicit PermutationMatrix(const Map<const IndicesType>& m) : idx_(m.size(), 1) {
    for (int k = 0; k < m.size(); ++k) idx_(k) = m.data()[k];
  }
  void setIdentity(int n) {
    idx_.resize(n, 1);
    for (int k = 0; k < n; ++k) idx_(k) = (vehidx_t)k;
  }
  int size() const { return idx_.size(); }
  int rows() const { return idx_.size(); }
  int cols() const { return idx_.size(); }
  IndicesType& indices() { return idx_; }
  const IndicesType& indices() const { return idx_; }
  PermutationMatrix transpose() const {  // the inverse
    PermutationMatrix t(size());
    for (int k = 0; k < size(); ++k) t.idx_(idx_(k)) = (vehidx_t)k;
    return t;
  }
  PermutationMatrix inverse() const { return transpose(); }

 private:
  IndicesType idx_;
};

class Vector3d {
 public:
  Vector3d() : v_{0.0, 0.0, 0.0} {}
  Vector3d(double x, double y, double z) : v_{x, y, z} {}
  static Vector3d Zero() { return Vector3d(); }
  double* data() { return v_; }
  const double* data() const { return v_; }
  double& operator()(int i) { return v_[i]; }
  double operator()(int i) const { return v_[i]; }
  double& x() { return v_[0]; }
  double& y() { return v_[1]; }
  double& z() { return v_[2]; }
  double x() const { return v_[0]; }
  double y() const { return v_[1]; }
  double z() const { return v_[2]; }
  int size() const { return 3; }

 private:
  double v_[3];
};

}  // namespace mini

using GainMat = mini::Matrix<double>;
using AdjMat = mini::Matrix<vehidx_t>;
using PtsMat = mini::Matrix<double>;
using AssignmentVec = mini::Matrix<vehidx_t>;
using AssignmentPerm = mini::PermutationMatrix;
using MatrixXd = mini::Matrix<double>;
using Matrix3Xd = mini::Matrix<double>;
using Vector3d = mini::Vector3d;
template <class M>
using Map = mini::Map<M>;
#else
// utils.h:25-30 exactly
using GainMat = Eigen::MatrixXd;
using AdjMat = Eigen::Matrix<vehidx_t, Eigen::Dynamic, Eigen::Dynamic>;
using PtsMat = Eigen::Matrix<double, Eigen::Dynamic, 3>;
using AssignmentVec = Eigen::Matrix<vehidx_t, Eigen::Dynamic, 1>;
using AssignmentPerm = Eigen::PermutationMatrix<Eigen::Dynamic, Eigen::Dynamic, vehidx_t>;
using MatrixXd = Eigen::MatrixXd;
using Matrix3Xd = Eigen::Matrix<double, 3, Eigen::Dynamic>;
using Vector3d = Eigen::Vector3d;
template <class M>
using Map = Eigen::Map<M>;
#endif

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
  using AssignmentPerm = amd::AssignmentPerm;
  using PtsMat = amd::PtsMat;
  using AdjMat = amd::AdjMat;
  /* auctioneer.h:31-34 */
  struct Bid {
    std::vector<float> price;
    std::vector<int> who;
  };
  using BidPtr = std::shared_ptr<Bid>;
  using BidConstPtr = std::shared_ptr<const Bid>;

  /* auctioneer.cpp:13-22: assignment initialised to identity */
  Auctioneer(vehidx_t vehid, uint8_t n, bool verbose = false)
      : n_(n), vehid_(vehid), verbose_(verbose) {
    if (n_ < 1 || vehid_ >= n_) throw std::runtime_error("Auctioneer: vehid >= n");
    P_.resize(n_);
    Pt_.resize(n_);
    for (int i = 0; i < n_; ++i) P_[i] = Pt_[i] = (vehidx_t)i;
  }

  /* auctioneer.h:59: the handler gets P (vehicle -> formation point) */
  void setNewAssignmentHandler(std::function<void(const AssignmentPerm&)> f) {
    handler_ = std::move(f);
  }
  /* C callback form: f(user, P, n). */
  void setNewAssignmentHandler(acl_new_assignment_fn f, void* user) {
    if (!f) { handler_ = nullptr; return; }
    handler_ = [f, user](const AssignmentPerm& P) {
      f(user, P.indices().data(), (int32_t)P.indices().size());
    };
  }
  /* Called once per auction with the final bid (see file header). */
  void setSendBidHandler(std::function<void(uint32_t, uint32_t, const BidConstPtr&)> f) {
    send_bid_ = std::move(f);
  }

  /* auctioneer.cpp:42-61: new formation; assignment reset to identity and the
   * next auction's result is adopted unconditionally. */
  void setFormation(const PtsMat& p, const AdjMat& adjmat) {
    if (p.rows() != n_ || p.cols() != 3 || adjmat.rows() != n_ || adjmat.cols() != n_)
      throw std::runtime_error("Auctioneer::setFormation: sizes do not match n");
    setFormationColMajor(p.data(), adjmat.data());
  }
  /* p column-major n x 3, adjmat column-major n x n */
  void setFormationColMajor(const double* p_colmajor, const uint8_t* adj_colmajor) {
    form_.upload(n_, p_colmajor, adj_colmajor, nullptr);
    form_p_ = detail::rows_xyz(n_, p_colmajor);
    adj_.assign(adj_colmajor, adj_colmajor + (size_t)n_ * n_);
    cbaa_max_iter_ = 2 * n_;  // n * diameter, diameter = 2 (auctioneer.cpp:50-51)
    reset_x();
    auction_open_ = false;
    formation_just_received_ = true;
    for (int i = 0; i < n_; ++i) P_[i] = Pt_[i] = (vehidx_t)i;
  }

  /* auctioneer.cpp:78-125 + 245-306: run the auction on snapshot q to
   * consensus and adopt this vehicle's result. */
  void start(const PtsMat& q) {
    if (q.rows() != n_ || q.cols() != 3) {
      last_status_ = ACL_ERR_INVALID_ARG;
      last_error_ = "Auctioneer::start: q is not n x 3";
      return;
    }
    startColMajor(q.data());
  }
  /* q column-major n x 3 */
  void startColMajor(const double* q_colmajor) {
    std::lock_guard<std::mutex> lock(auction_mtx_);
    if (form_.n != n_) {
      last_status_ = ACL_ERR_INVALID_ARG;
      last_error_ = "Auctioneer::start before setFormation";
      return;
    }
    if (exchange_) {
      start_exchange(q_colmajor);
      return;
    }
    AuctionOut r;
    try {
      r = run_auction(q_colmajor);
      last_status_ = ACL_OK;
      last_error_.clear();
    } catch (const std::exception& e) {
      last_status_ = ACL_ERR_HIP;
      last_error_ = e.what();
      auction_open_ = false;
      return;
    }
    auction_open_ = false;
    // The user's handlers run outside the GPU error channel: the vehicle
    // adopts its result first (auctioneer.cpp:250-295, which notifies the
    // new-assignment handler), then the final bid is published; an exception
    // either handler throws reaches the caller, as it would out of the
    // reference's processBid, and is not reported as a GPU failure.
    finish(r.who);
    if (send_bid_) send_bid_((uint32_t)auctionid_, (uint32_t)(2 * n_), finalBid(r.q, r.who, r.Rt));
  }
  /* the outcome of the last start(): ACL_OK, or why no auction ran
   * (lastError() says what); in exchange mode also a tally that failed or a
   * malformed bid that processBid dropped (ACL_ERR_INVALID_ARG) */
  acl_status_t lastStatus() const { return last_status_; }
  const std::string& lastError() const { return last_error_; }

 private:
  struct AuctionOut {
    std::vector<double> q;     // the snapshot, xyz rows
    std::vector<uint16_t> who; // this vehicle's final table: task -> vehicle
    std::vector<double> Rt;    // every vehicle's alignment (R, t)
  };
  AuctionOut run_auction(const double* q_colmajor) {
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
    d_rt_.reserve((size_t)n * 6 * 8);
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
    a.align_Rt = d_rt_.as<double>();
    a.workspace = d_ws_.get();
    acl_default_cntrl_gains(&a.cntrl);
    acl_default_safety_params(&a.safety);
    a.early_exit = 1;
    a.do_control = 0;
    detail::check(acl_solve_batch(&F, &a, nullptr));
    std::vector<uint16_t> who(n);  // this vehicle's final table: task -> vehicle
    std::vector<double> Rt((size_t)n * 6);
    detail::check(acl_memcpy_d2h(who.data(), d_who_.as<uint16_t>() + (size_t)vehid_ * n,
                                 (size_t)n * 2, nullptr));
    detail::check(acl_memcpy_d2h(Rt.data(), d_rt_.get(), Rt.size() * 8, nullptr));
    detail::check(acl_stream_synchronize(nullptr));
    return AuctionOut{q, std::move(who), std::move(Rt)};
  }

  /* The final bid of this vehicle: who[j] (-1 = none) and price[j] = the
   * holder's getPrice for task j (auctioneer.cpp:546-549), from the holder's
   * alignment (R, t) applied to formation point j as alignFormation does
   * (R p + t, z row identity, auctioneer.cpp:400-414): the same f64
   * operations, so the float equals the holder's bid bit for bit. */
  BidConstPtr finalBid(const std::vector<double>& q, const std::vector<uint16_t>& who,
                       const std::vector<double>& Rt) const {
    const int n = n_;
    auto bid = std::make_shared<Bid>();
    bid->price.assign(n, 0.0f);
    bid->who.assign(n, -1);
    for (int j = 0; j < n; ++j) {
      const unsigned w = who[j];
      if (w >= (unsigned)n) continue;
      const double* o = &Rt[(size_t)6 * w];
      const double px = form_p_[(size_t)3 * j], py = form_p_[(size_t)3 * j + 1],
                   pz = form_p_[(size_t)3 * j + 2];
      const double ax = ((o[0] * px + o[1] * py) + 0.0 * pz) + o[4];
      const double ay = ((o[2] * px + o[3] * py) + 0.0 * pz) + o[5];
      const double az = ((0.0 * px + 0.0 * py) + 1.0 * pz) + 0.0;
      const double dx = q[(size_t)3 * w] - ax, dy = q[(size_t)3 * w + 1] - ay,
                   dz = q[(size_t)3 * w + 2] - az;
      bid->price[j] = (float)(1.0 / (std::sqrt((dx * dx + dy * dy) + dz * dz) + 1e-8));
      bid->who[j] = (int)w;
    }
    return bid;
  }

 public:

  /* Exchange mode (see the file header): off by default, where the whole
   * consensus runs inside start(). Set it before the first start(). */
  void setBidExchange(bool on) {
    std::lock_guard<std::mutex> lock(auction_mtx_);
    exchange_ = on;
  }
  bool bidExchange() const { return exchange_; }

  /* auctioneer.cpp:124-135. Default mode: accepted and dropped (the
   * consensus ran inside start()); exchange mode: queued for tick(). */
  void enqueueBid(vehidx_t vehid, uint32_t auctionid, uint32_t iter, const Bid& bid) {
    std::lock_guard<std::mutex> lock(queue_mtx_);
    if (exchange_) rxbids_.push_back(BidPkt{vehid, auctionid, iter, bid});
  }
  /* auctioneer.cpp:139-160: exchange mode processes the oldest queued bid
   * (processBid, :182-306) while an auction is open. */
  void tick() {
    std::lock_guard<std::mutex> lock(auction_mtx_);
    if (!exchange_ || !auction_open_) return;
    BidPkt pkt;
    {
      std::lock_guard<std::mutex> qlock(queue_mtx_);
      if (rxbids_.empty()) return;
      pkt = rxbids_.front();
      rxbids_.erase(rxbids_.begin());
    }
    processBid(pkt);
  }
  /* bids waiting for tick() (exchange mode) */
  size_t queuedBids() {
    std::lock_guard<std::mutex> lock(queue_mtx_);
    return rxbids_.size();
  }

  /* auctioneer.cpp:65-74 */
  void flush() {
    reset_x();
    bids_zero_.clear();
    {
      std::lock_guard<std::mutex> lock(queue_mtx_);
      rxbids_.clear();
    }
    auction_open_ = false;
    invalid_assignment_ = false;
  }

  /* auctioneer.h:103-104: P (vehicle -> formation point), Pt = P^-1 */
  AssignmentPerm getAssignment() const { return toPerm(P_); }
  AssignmentPerm getInvAssignment() const { return toPerm(Pt_); }
  /* auctioneer.h:107: the "backdoor" override, Pt = P^T */
  void setAssignment(const AssignmentPerm& P) { setAssignmentIndices(P.indices().data()); }

  /* the same as plain index vectors */
  const std::vector<vehidx_t>& getAssignmentIndices() const { return P_; }
  const std::vector<vehidx_t>& getInvAssignmentIndices() const { return Pt_; }
  void setAssignmentIndices(const vehidx_t* P) {
    for (int i = 0; i < n_; ++i) {
      P_[i] = P[i];
      Pt_[P[i]] = (vehidx_t)i;
    }
  }

  bool isIdle() const { return !auction_open_; }
  bool didConvergeOnInvalidAssignment() const { return invalid_assignment_; }
  int auctionId() const { return auctionid_; }

 private:
  static AssignmentPerm toPerm(const std::vector<vehidx_t>& v) {
    AssignmentPerm perm((int)v.size());
    for (size_t i = 0; i < v.size(); ++i) perm.indices()((int)i) = v[i];
    return perm;
  }

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
    if (handler_) handler_(toPerm(P_));
  }

  // ---- exchange mode (auctioneer.cpp:78-125,182-306,419-465) ----
  struct BidPkt {
    vehidx_t vehid;
    uint32_t auctionid, iter;
    Bid bid;
  };

  /* reset (auctioneer.cpp:448-465) */
  void reset_x() {
    auction_open_ = false;
    biditer_ = 0;
    bid_.price.assign(n_, 0.0f);
    bid_.who.assign(n_, -1);
    bids_curr_.clear();
    bids_next_.clear();
  }

  void notifySendBid() {
    if (send_bid_) send_bid_((uint32_t)auctionid_, (uint32_t)biditer_, std::make_shared<const Bid>(bid_));
  }

  /* start (auctioneer.cpp:78-120): alignment on the GPU, the START bid */
  void start_exchange(const double* q_colmajor) {
    reset_x();
    bids_curr_ = bids_zero_;
    bids_zero_.clear();
    try {
      const AuctionOut r = run_auction(q_colmajor);  // this vehicle's align_Rt row
      q_self_[0] = r.q[(size_t)3 * vehid_];
      q_self_[1] = r.q[(size_t)3 * vehid_ + 1];
      q_self_[2] = r.q[(size_t)3 * vehid_ + 2];
      std::copy(r.Rt.begin() + (size_t)6 * vehid_, r.Rt.begin() + (size_t)6 * vehid_ + 6, rt_self_);
      step(true);
      last_status_ = ACL_OK;
      last_error_.clear();
    } catch (const std::exception& e) {
      last_status_ = ACL_ERR_HIP;
      last_error_ = e.what();
      reset_x();
      return;
    }
    auction_open_ = true;  // (run_auction counted the auction id)
    notifySendBid();
  }

  /* bidIterComplete (auctioneer.cpp:419-437): a bid from every neighbour of
   * this vehicle's formation point under its own assignment */
  bool bidIterComplete() const {
    const int i = P_[vehid_];
    for (int j = 0; j < n_; ++j)
      if (adj_[(size_t)j * n_ + i] && bids_curr_.find(Pt_[j]) == bids_curr_.end()) return false;
    return true;
  }

  /* processBid (auctioneer.cpp:182-306) */
  void processBid(const BidPkt& pkt) {
    if ((int)pkt.bid.price.size() != n_ || (int)pkt.bid.who.size() != n_) {
      // a malformed bid (the reference would index past its tables): dropped
      last_status_ = ACL_ERR_INVALID_ARG;
      last_error_ = "Auctioneer: dropped a bid whose tables are not n long";
      return;
    }
    if (verbose_)
      std::cout << "A" << auctionid_ << "B" << biditer_ << ": Processing a" << pkt.auctionid
                << "b" << pkt.iter << " from " << static_cast<int>(pkt.vehid) << std::endl;
    if (pkt.iter == 0) bids_zero_.insert({pkt.vehid, pkt.bid});
    if (pkt.iter == (uint32_t)biditer_) bids_curr_.insert({pkt.vehid, pkt.bid});
    else if (pkt.iter == (uint32_t)biditer_ + 1) bids_next_.insert({pkt.vehid, pkt.bid});
    else if (verbose_)
      std::cout << "!! Threw away a" << pkt.auctionid << "b" << pkt.iter << " from "
                << static_cast<int>(pkt.vehid) << std::endl;
    if (!bidIterComplete()) return;
    try {
      step(false);  // updateTaskAssignment, then selectTaskAssignment if outbid
    } catch (const std::exception& e) {
      last_status_ = ACL_ERR_HIP;
      last_error_ = e.what();
      reset_x();
      return;
    }
    ++biditer_;
    bids_curr_ = bids_next_;
    bids_next_.clear();
    if (biditer_ == 1) bids_zero_.clear();
    if (biditer_ >= cbaa_max_iter_) {  // hasReachedConsensus (:442-444)
      std::vector<uint16_t> who(n_);
      for (int j = 0; j < n_; ++j)
        who[j] = (bid_.who[j] >= 0 && bid_.who[j] < n_) ? (uint16_t)bid_.who[j] : (uint16_t)0xFFFF;
      finish(who);  // (:256-292) adoption, the new-assignment handler
      reset_x();    // (:295) idle for the next auction
    } else {
      notifySendBid();
    }
  }

  /* One tally of this vehicle on the GPU (acl_cbaa_step_batch, V = 1): the
   * START bid, or the candidates = bids_curr_ with its own bid inserted
   * (:475, std::map order) */
  void step(bool start) {
    const int n = n_;
    std::vector<int32_t> cv;
    std::vector<float> cp;
    std::vector<int32_t> cw;
    if (!start) {
      std::map<vehidx_t, Bid> cand = bids_curr_;
      cand.insert({vehid_, bid_});
      for (const auto& kv : cand) {
        if ((int)kv.second.price.size() != n || (int)kv.second.who.size() != n)
          throw std::runtime_error("Auctioneer: a bid's tables are not n long");
        cv.push_back((int32_t)kv.first);
        cp.insert(cp.end(), kv.second.price.begin(), kv.second.price.end());
        cw.insert(cw.end(), kv.second.who.begin(), kv.second.who.end());
      }
    }
    const int K = (int)cv.size();
    // one staging image each way (one copy up, one down): doubles first,
    // then the table (price, who) and the outputs (task, flags) contiguous,
    // then the small ints and the candidates
    const size_t o_q = 0, o_rt = 24, o_price = 72, o_who = o_price + (size_t)4 * n,
                 o_out = o_who + (size_t)4 * n, o_i = o_out + 8, o_off = o_i + 8, o_st = o_off + 8,
                 o_cv = o_st + 8, o_cp = o_cv + (size_t)4 * K,
                 o_cw = o_cp + (size_t)4 * K * n, total = o_cw + (size_t)4 * K * n;
    std::vector<unsigned char> h(total, 0);
    const int32_t ids[2] = {0, (int32_t)vehid_};  // fidx, vehid
    const int32_t off[2] = {0, K};
    std::memcpy(&h[o_q], q_self_, 24);
    std::memcpy(&h[o_rt], rt_self_, 48);
    std::memcpy(&h[o_price], bid_.price.data(), (size_t)4 * n);
    for (int j = 0; j < n; ++j) {
      const int32_t w = bid_.who[j];
      std::memcpy(&h[o_who + (size_t)4 * j], &w, 4);
    }
    std::memcpy(&h[o_i], ids, 8);
    std::memcpy(&h[o_off], off, 8);
    h[o_st] = start ? 1 : 0;
    if (K) {
      std::memcpy(&h[o_cv], cv.data(), (size_t)4 * K);
      std::memcpy(&h[o_cp], cp.data(), cp.size() * 4);
      std::memcpy(&h[o_cw], cw.data(), cw.size() * 4);
    }
    x_stage_.upload(h.data(), total);
    unsigned char* d = x_stage_.as<unsigned char>();
    acl_cbaa_step_args_t a;
    std::memset(&a, 0, sizeof(a));
    a.V = 1;
    a.K = K;
    a.fidx = reinterpret_cast<const int32_t*>(d + o_i);
    a.vehid = reinterpret_cast<const int32_t*>(d + o_i) + 1;
    a.q = reinterpret_cast<const double*>(d + o_q);
    a.Rt = reinterpret_cast<const double*>(d + o_rt);
    a.start = d + o_st;
    a.price = reinterpret_cast<float*>(d + o_price);
    a.who = reinterpret_cast<int32_t*>(d + o_who);
    a.cand_off = reinterpret_cast<const int32_t*>(d + o_off);
    a.cand_vehid = K ? reinterpret_cast<const int32_t*>(d + o_cv) : nullptr;
    a.cand_price = K ? reinterpret_cast<const float*>(d + o_cp) : nullptr;
    a.cand_who = K ? reinterpret_cast<const int32_t*>(d + o_cw) : nullptr;
    a.task = reinterpret_cast<int32_t*>(d + o_out);
    a.flags = reinterpret_cast<int32_t*>(d + o_out) + 1;
    const acl_formations_t F = form_.table();
    detail::check(acl_cbaa_step_batch(&F, &a, nullptr));
    detail::check(acl_memcpy_d2h(&h[o_price], d + o_price, o_i - o_price, nullptr));
    detail::check(acl_stream_synchronize(nullptr));
    int32_t out[2];
    std::memcpy(out, &h[o_out], 8);
    if (out[1] & ACL_CBAA_BAD_INPUT) throw std::runtime_error("acl_cbaa_step_batch: bad input");
    std::memcpy(bid_.price.data(), &h[o_price], (size_t)4 * n);
    std::vector<int32_t> who(n);
    std::memcpy(who.data(), &h[o_who], (size_t)4 * n);
    bid_.who.assign(who.begin(), who.end());
  }

  int n_;
  vehidx_t vehid_;
  bool verbose_;
  std::atomic<bool> exchange_{false};  // read by enqueueBid without the auction mutex
  int biditer_ = 0, cbaa_max_iter_ = 0;
  Bid bid_;
  std::map<vehidx_t, Bid> bids_zero_, bids_curr_, bids_next_;
  std::vector<BidPkt> rxbids_;  // FIFO (std::queue in the reference)
  std::vector<uint8_t> adj_;    // AdjMat, column-major
  double q_self_[3] = {0.0, 0.0, 0.0}, rt_self_[6] = {1.0, 0.0, 0.0, 1.0, 0.0, 0.0};
  detail::DeviceBuffer x_stage_;  // acl_cbaa_step_batch's staging image (step())
  std::vector<vehidx_t> P_, Pt_;
  int auctionid_ = 0;
  bool auction_open_ = false;
  bool invalid_assignment_ = false;
  bool formation_just_received_ = false;
  std::mutex queue_mtx_, auction_mtx_;
  std::function<void(const AssignmentPerm&)> handler_;
  std::function<void(uint32_t, uint32_t, const BidConstPtr&)> send_bid_;
  acl_status_t last_status_ = ACL_OK;
  std::string last_error_;
  std::vector<double> form_p_;  // formation points, xyz rows (final bids)
  detail::DeviceFormation form_;
  detail::DeviceBuffer d_q_, d_pin_, d_fidx_, d_pout_, d_status_, d_who_, d_rt_, d_ws_;
};

// ============================================================================
// DistCntrl (distcntrl.h:23-66, distcntrl.cpp:20-102)
// ============================================================================

class DistCntrl {
 public:
  using AssignmentPerm = amd::AssignmentPerm;
  using PtsMat = amd::PtsMat;

  /* distcntrl.h:26-34 (column-major Eigen storage); dstar_* are filled by
   * setFormation as the reference does */
  struct Formation {
    std::string name;
    AdjMat adjmat;   // n x n
    GainMat gains;   // 3n x 3n
    PtsMat qdes;     // n x 3
    MatrixXd dstar_xy;
    MatrixXd dstar_z;
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
    if (!f || f->qdes.rows() != n || f->qdes.cols() != 3 || f->adjmat.rows() != n ||
        f->adjmat.cols() != n || f->gains.rows() != 3 * n || f->gains.cols() != 3 * n)
      throw std::runtime_error("DistCntrl::setFormation: formation sizes do not match n");
    formation_ = f;
    f->dstar_xy.resize(n, n);
    f->dstar_z.resize(n, n);
    pdist(f->qdes.data(), 0, 2, f->dstar_xy.data());
    pdist(f->qdes.data(), 2, 3, f->dstar_z.data());
    form_.upload(n, f->qdes.data(), f->adjmat.data(), f->gains.data());
  }

  /* distcntrl.cpp:39-42; P: vehicle -> formation point. */
  void setAssignment(const AssignmentPerm& P) { setAssignmentIndices(P.indices().data()); }
  void setAssignmentIndices(const vehidx_t* P) {
    for (int i = 0; i < n_; ++i) P_[i] = P[i];
  }

  /* distcntrl.cpp:46-102: u for this vehicle from the snapshot q_veh
   * (vehicle space, n x 3) and its velocity. */
  Vector3d compute(const PtsMat& q_veh, const Vector3d vel) {
    if (q_veh.rows() != n_ || q_veh.cols() != 3)
      throw std::runtime_error("DistCntrl::compute: q_veh is not n x 3");
    Vector3d u;
    computeColMajor(q_veh.data(), vel.data(), u.data());
    return u;
  }
  /* q_veh column-major n x 3, vel[3] -> u[3] */
  void computeColMajor(const double* q_veh_colmajor, const double vel[3], double u[3]) {
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

 private:
  // squareform(pdist(M)) over columns [c0, c1) of the n x 3 matrix, by the
  // reference's |x|^2 + |y|^2 - 2 x'y identity (utils.h:140-146); D is n x n
  // column-major
  void pdist(const double* M, int c0, int c1, double* D) const {
    const int n = n_;
    std::vector<double> N(n, 0.0);
    for (int i = 0; i < n; ++i)
      for (int c = c0; c < c1; ++c) N[i] += M[(size_t)c * n + i] * M[(size_t)c * n + i];
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
    /* not in solver.h: the 2-D complement basis (acl_admm_params_t.basis).
     * The complex-structured basis makes solve() meet the block-structure
     * and zero-block properties test_admm.cpp:84-187 asserts; set
     * ACL_ADMM_BASIS_LINPACK for the codegen ADMM's exact gains. */
    int basis = ACL_ADMM_BASIS_COMPLEX;
  };

  Solver() : Solver(Params()) {}
  explicit Solver(const Params& params) : params_(params) {}

  /* solver.h:38: gains (3n x 3n) for the points (3 x n) and adjacency (n x n) */
  MatrixXd solve(const Matrix3Xd& pts, const MatrixXd& adj) {
    const int n = (int)pts.cols();
    if (pts.rows() != 3 || adj.rows() != n || adj.cols() != n)
      throw std::runtime_error("admm::Solver::solve: pts must be 3 x n and adj n x n");
    MatrixXd A(3 * n, 3 * n);
    solveColMajor(n, pts.data(), adj.data(), A.data());
    return A;
  }

  /* pts column-major 3 x n, adj column-major n x n f64, gains out
   * column-major 3n x 3n */
  void solveColMajor(int n, const double* pts_3xn, const double* adj_nxn, double* gains_out) {
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
    p.basis = (int32_t)params_.basis;
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

  /* ADMM iteration counts of the last solve (2-D, 1-D). */
  int iterations2d() const { return iters_[0]; }
  int iterations1d() const { return iters_[1]; }

 private:
  Params params_;
  int32_t iters_[2] = {0, 0};
  detail::DeviceBuffer d_pts_, d_adj_, d_gains_, d_iters_;
};

}  // namespace admm

// ============================================================================
// ADMM (aclswarm/include/aclswarm/admm.h:27-40, src/admm.cpp:12-55): the
// wrapper of the MATLAB-Coder ADMMGainDesign3D -- codegen semantics (the
// LINPACK complement basis, acl_admm_params_t defaults) and the wrapper's
// |a| <= 1e-10 zeroing (admm.cpp:50, applied by acl_admm_solve_batch).
// ============================================================================
class ADMM {
 public:
  explicit ADMM(const size_t n) : solver_(params_for_codegen()) { (void)n; }

  /* admm.cpp:34-55: p is n x 3 (PtsMat), adjmat n x n (AdjMat) */
  GainMat calculateFormationGains(const PtsMat& p, const AdjMat& adjmat) {
    return solver_.solve(p.transpose(), adjmat.template cast<double>());
  }

 private:
  static admm::Solver::Params params_for_codegen() {
    admm::Solver::Params prm;
    prm.basis = ACL_ADMM_BASIS_LINPACK;
    return prm;
  }
  admm::Solver solver_;
};

}  // namespace amd
}  // namespace aclswarm
}  // namespace acl

#endif  // ACLSWARM_AMD_HPP
