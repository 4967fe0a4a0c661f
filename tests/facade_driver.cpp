// facade_driver.cpp -- exercises include/aclswarm_amd.hpp the way the
// reference's CoordinationROS uses its objects (coordination_ros.cpp:115-129,
// 176-205, 336-378): one Auctioneer and one DistCntrl per vehicle, one
// admm::Solver. Built by aclswarm_amd/build.py into
// aclswarm_amd/lib/libfacade_driver.so (a library, loaded by ctypes into the
// test process: no child process is started after the GPU is initialised);
// tests/test_gpu_facade.py calls facade_run(in, out) on a case file and
// checks what it writes against the CPU restatement.
//
// input  (little endian): i32 n; f64 p[n*3] (PtsMat, column-major);
//        u8 adj[n*n] (AdjMat, column-major); f64 gains[9n^2] (GainMat,
//        column-major); f64 q[n*3] (column-major); f64 vel[n][3];
//        u8 P_in[n]; i32 m; f64 pts[3*m] (3 x m column-major); f64 adjf[m*m]
// output: per vehicle v: u8 P[n], u8 invalid, u8 handler_calls;
//         f64 u[n][3]; i32 iters[2]; f64 A[9m^2] (column-major)
#include <stdio.h>

#include <memory>
#include <vector>

#include "aclswarm_amd.hpp"

namespace amd = acl::aclswarm::amd;

template <class T>
static void rd(FILE* f, T* p, size_t n) {
  if (n && fread(p, sizeof(T), n, f) != n) throw std::runtime_error("short read");
}
template <class T>
static void wr(FILE* f, const T* p, size_t n) {
  if (n && fwrite(p, sizeof(T), n, f) != n) throw std::runtime_error("short write");
}

static void on_assignment(void* user, const amd::vehidx_t*, int32_t) {
  ++*static_cast<int*>(user);
}

extern "C" int facade_run(const char* in_path, const char* out_path) {
  try {
    FILE* in = fopen(in_path, "rb");
    if (!in) throw std::runtime_error("cannot open input");
    int32_t n = 0, m = 0;
    rd(in, &n, 1);
    std::vector<double> p(3 * n), gains((size_t)9 * n * n), q(3 * n), vel(3 * n);
    std::vector<uint8_t> adj((size_t)n * n), Pin(n);
    rd(in, p.data(), p.size());
    rd(in, adj.data(), adj.size());
    rd(in, gains.data(), gains.size());
    rd(in, q.data(), q.size());
    rd(in, vel.data(), vel.size());
    rd(in, Pin.data(), Pin.size());
    rd(in, &m, 1);
    std::vector<double> pts(3 * m), adjf((size_t)m * m);
    rd(in, pts.data(), pts.size());
    rd(in, adjf.data(), adjf.size());
    fclose(in);

    FILE* out = fopen(out_path, "wb");
    if (!out) throw std::runtime_error("cannot open output");

    // auction: every vehicle's Auctioneer on the same snapshot
    std::vector<std::vector<amd::vehidx_t>> Pveh(n);
    for (int v = 0; v < n; ++v) {
      amd::Auctioneer auc((amd::vehidx_t)v, (uint8_t)n);
      int calls = 0;
      auc.setNewAssignmentHandler(&on_assignment, &calls);
      auc.setFormation(p.data(), adj.data());
      auc.setAssignment(Pin.data());
      auc.start(q.data());
      if (!auc.isIdle()) throw std::runtime_error("auction still open after start");
      Pveh[v] = auc.getAssignment();
      const std::vector<amd::vehidx_t> Pt = auc.getInvAssignment();
      for (int i = 0; i < n; ++i)
        if (Pt[Pveh[v][i]] != i) throw std::runtime_error("getInvAssignment is not P^-1");
      const uint8_t inv = auc.didConvergeOnInvalidAssignment() ? 1 : 0;
      const uint8_t nc = (uint8_t)calls;
      wr(out, Pveh[v].data(), n);
      wr(out, &inv, 1);
      wr(out, &nc, 1);
    }

    // control: each vehicle's DistCntrl with the assignment it adopted
    auto form = std::make_shared<amd::DistCntrl::Formation>();
    form->name = "facade";
    form->adjmat = adj;
    form->gains = gains;
    form->qdes = p;
    amd::DistCntrl::Gains g{};
    {
      acl_cntrl_gains_t d;
      acl_default_cntrl_gains(&d);
      g = {d.K1_xy, d.K2_xy, d.K1_z, d.K2_z, d.e_xy_thr, d.e_z_thr, d.kp, d.kd};
    }
    for (int v = 0; v < n; ++v) {
      amd::DistCntrl ctl((amd::vehidx_t)v, (uint8_t)n);
      ctl.setGains(g);
      ctl.setFormation(form);
      ctl.setAssignment(Pveh[v].data());
      double u[3];
      ctl.compute(q.data(), &vel[3 * v], u);
      wr(out, u, 3);
    }
    if (form->dstar_xy.size() != (size_t)n * n) throw std::runtime_error("dstar not filled");

    // ADMM gain design
    int32_t its[2] = {0, 0};
    std::vector<double> A((size_t)9 * m * m);
    if (m > 0) {
      amd::admm::Solver solver;
      solver.solve(m, pts.data(), adjf.data(), A.data());
      its[0] = solver.iterations2d();
      its[1] = solver.iterations1d();
    }
    wr(out, its, 2);
    wr(out, A.data(), A.size());
    fclose(out);
  } catch (const std::exception& e) {
    fprintf(stderr, "facade_driver: %s\n", e.what());
    return 1;
  }
  return 0;
}
