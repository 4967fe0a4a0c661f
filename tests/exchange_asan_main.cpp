// exchange_asan_main.cpp -- the facade's exchange-mode host protocol
// (include/aclswarm_amd.hpp: queues, iteration buckets, the staging image of
// each acl_cbaa_step_batch call) under host AddressSanitizer /
// UndefinedBehaviorSanitizer: fleets of n exchange-mode Auctioneers on a bus
// (each sender's bids in order, senders interleaved), a second auction from
// the adopted assignments, a restart while busy and a flush. Built and run by
// scripts/facade_asan.sh (g++ -fsanitize=address,undefined on the host code
// only; the GPU kernels are the in-tree library's). Exit 0: in every auction
// all vehicles adopted one and the same valid assignment (or all flagged it
// invalid), and no sanitizer report.
#include <stdio.h>

#include <algorithm>
#include <cmath>
#include <memory>
#include <vector>

#include "aclswarm_amd.hpp"

namespace amd = acl::aclswarm::amd;

namespace {

struct Msg {
  int from;
  uint32_t a, it;
  amd::Auctioneer::Bid b;
};

struct Fleet {
  int n;
  amd::PtsMat p, q;
  amd::AdjMat adj;
  std::vector<Msg> bus;
  std::vector<std::unique_ptr<amd::Auctioneer>> v;
  unsigned s;

  Fleet(int n_, unsigned seed) : n(n_), p(n_, 3), q(n_, 3), adj(n_, n_), s(seed) {
    // a ring with chords (connected), points on a circle, a scrambled start
    for (int i = 0; i < n; ++i) {
      p(i, 0) = 10.0 * std::cos(6.283185307179586 * i / n);
      p(i, 1) = 10.0 * std::sin(6.283185307179586 * i / n);
      p(i, 2) = 1.0 + 0.1 * (i % 3);
      q(i, 0) = 3.0 * ((i * 7 + 3) % n);
      q(i, 1) = 2.0 * ((i * 5 + 1) % n);
      q(i, 2) = 1.0;
      for (int j = 0; j < n; ++j) adj(i, j) = 0;
    }
    for (int i = 0; i < n; ++i)
      for (int d : {1, 2, 5}) {
        const int j = (i + d) % n;
        if (j != i) adj(i, j) = adj(j, i) = 1;
      }
    v.resize(n);
    for (int k = 0; k < n; ++k) {
      v[k].reset(new amd::Auctioneer((amd::vehidx_t)k, (uint8_t)n, false));
      v[k]->setBidExchange(true);
      v[k]->setFormation(p, adj);
      v[k]->setSendBidHandler(
          [this, k](uint32_t a, uint32_t it, const amd::Auctioneer::BidConstPtr& b) {
            bus.push_back(Msg{k, a, it, *b});
          });
    }
  }
  unsigned rnd(unsigned m) {
    s = s * 1664525u + 1013904223u;
    return (s >> 8) % m;
  }
  // vehicle u receives the sender's bids iff the sender sits at a neighbour
  // of u's formation point under u's own assignment (connectToNeighbors)
  bool subscribes(int u, int from) const {
    const auto& P = v[u]->getAssignmentIndices();
    const auto& Pt = v[u]->getInvAssignmentIndices();
    for (int j = 0; j < n; ++j)
      if (adj(P[u], j) && Pt[j] == from) return true;
    return false;
  }
  // deliver until quiet; `budget` > 0 stops after that many deliveries
  void pump(long budget) {
    for (long g = 0; g < 10000000 && (budget <= 0 || g < budget); ++g) {
      if (!bus.empty()) {
        size_t m = rnd((unsigned)bus.size());
        for (size_t k = 0; k < m; ++k)
          if (bus[k].from == bus[m].from) {
            m = k;
            break;
          }
        const Msg msg = bus[m];
        bus.erase(bus.begin() + (long)m);
        for (int u = 0; u < n; ++u)
          if (u != msg.from && subscribes(u, msg.from))
            v[u]->enqueueBid((amd::vehidx_t)msg.from, msg.a, msg.it, msg.b);
      }
      // (a vehicle that adopted may hold late bids of the old auction from a
      // vehicle it subscribes to under its new assignment, as a ROS node
      // would; they wait in its queue for its next start, where iterations
      // other than 0 and 1 are thrown away)
      bool busy = !bus.empty();
      for (int k = 0; k < n && !busy; ++k) busy = !v[k]->isIdle() && v[k]->queuedBids() > 0;
      if (!busy) return;
      for (int k = 0; k < n; ++k) v[k]->tick();
    }
  }
  // every vehicle idle, and all adopted one valid assignment or all invalid
  bool consistent(int skip_status = -1) const {
    int invalid = 0;
    for (int k = 0; k < n; ++k) {
      if (!v[k]->isIdle() || (k != skip_status && v[k]->lastStatus() != ACL_OK)) return false;
      invalid += v[k]->didConvergeOnInvalidAssignment() ? 1 : 0;
    }
    if (invalid) return invalid == n;
    const auto& P0 = v[0]->getAssignmentIndices();
    std::vector<int> seen(n, 0);
    for (int k = 0; k < n; ++k) {
      if (v[k]->getAssignmentIndices() != P0 || P0[k] >= n || seen[P0[k]]++) return false;
    }
    return true;
  }
};

int check(bool ok, const char* what, int n) {
  if (!ok) fprintf(stderr, "exchange_asan: %s failed at n = %d\n", what, n);
  return ok ? 0 : 1;
}

}  // namespace

int main() {
  int bad = 0;
  for (int n : {6, 13, 40}) {
    Fleet f(n, 17u + (unsigned)n);
    for (auto& a : f.v) a->start(f.q);
    f.pump(0);
    bad += check(f.consistent(), "first auction", n);
    for (auto& a : f.v) a->start(f.q);  // the next auction from the adopted assignments
    // a malformed bid (tables of the wrong length) is dropped, not tallied
    amd::Auctioneer::Bid junk;
    junk.price.assign(3, 1.0f);
    junk.who.assign(5, 0);
    f.v[0]->enqueueBid(1, 2, 0, junk);
    f.pump(0);
    bad += check(f.consistent(0), "second auction", n);
    bad += check(f.v[0]->lastStatus() == ACL_ERR_INVALID_ARG, "malformed bid dropped", n);
    for (auto& a : f.v) a->start(f.q);  // restart while busy (autoauctionCb, :355-358)
    f.pump(3 * n);
    for (auto& a : f.v) a->start(f.q);
    f.pump(0);
    bad += check(f.consistent(), "restarted auction", n);
    for (auto& a : f.v) a->flush();  // flush clears the queue and the flag
    for (auto& a : f.v) bad += check(a->queuedBids() == 0 && a->isIdle(), "flush", n);
  }
  if (!bad) printf("exchange_asan: ok\n");
  return bad ? 1 : 0;
}
