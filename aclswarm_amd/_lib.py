"""Loader for the native engine library (libaclswarm_amd.so, built in-tree).

There is no fallback: if the HIP library is missing the import of any compute
entry point raises. Build it with `python -c "import __graft_entry__ as g;
g.build()"` (or `python -m aclswarm_amd.build`).
"""
import ctypes as ct
import os

import numpy as np

# ACLSWARM_AMD_LIB points at another build of the same library (kernel
# experiments); the default is the in-tree build.
LIB_PATH = os.environ.get("ACLSWARM_AMD_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "lib", "libaclswarm_amd.so")

ACL_OK = 0

FLAG_VALID = 0x01
FLAG_AGREE = 0x02
FLAG_CHANGED = 0x04
FLAG_NONFINITE = 0x08
FLAG_BAD_INPUT = 0x10
FLAG_CA_ACTIVE = 0x20
ABI_VERSION = 11  # include/aclswarm_amd.h ACL_ABI_VERSION
FLAG_FRAGILE = 0x40
FRAGILE_MARGIN = 1e-6

STATUS_DTYPE = np.dtype([("flags", "<u4"), ("eff_rounds", "<u2"),
                         ("rounds", "<u2"), ("n_invalid", "<u2"),
                         ("n_ca", "<u2"), ("margin", "<f4")])

# every symbol include/aclswarm_amd.h declares
EXPORTS = (
    "acl_default_cntrl_gains", "acl_default_safety_params", "acl_default_admm_params",
    "acl_formations_init", "acl_max_vehicles", "acl_abi_version", "acl_solve_workspace_bytes", "acl_solve_batch", "acl_swarm_stats", "acl_count_edges", "acl_pack_adjacency",
    "acl_pack_gains", "acl_gain_planes", "acl_pack_gains_planes", "acl_tile_gains", "acl_admm_solve_batch", "acl_device_count", "acl_set_device",
    "acl_control_batch", "acl_write_assignment_log", "acl_read_assignment_log",
    "acl_hungarian_batch", "acl_cbaa_step_batch",
    "acl_default_episode_params", "acl_episode_workspace_bytes", "acl_episode_batch",
    "acl_default_trial_params", "acl_trial_workspace_bytes", "acl_trial_init", "acl_trial_batch",
    "acl_generate_formation_groups",
    "acl_malloc", "acl_free", "acl_memcpy_h2d", "acl_memcpy_d2h", "acl_memset",
    "acl_stream_synchronize", "acl_last_error",
)


class CntrlGains(ct.Structure):
    """DistCntrl::Gains (aclswarm/include/aclswarm/distcntrl.h:36-45)."""
    _fields_ = [(n, ct.c_double) for n in
                ("K1_xy", "K2_xy", "K1_z", "K2_z", "e_xy_thr", "e_z_thr", "kp", "kd")]


class SafetyParams(ct.Structure):
    """Safety velocity/avoidance parameters (aclswarm/src/safety.cpp:49-52)."""
    _fields_ = [(n, ct.c_double) for n in
                ("max_vel_xy", "max_vel_z", "d_avoid_thresh", "r_keep_out")]


class AdmmParams(ct.Structure):
    """admm::Params (aclswarm/lib/admm/include/admm/solver.h:18-31)."""
    _fields_ = [("verbose", ct.c_int32), ("thrSparseZero", ct.c_double),
                ("thrPlanar", ct.c_double), ("epsEig", ct.c_double),
                ("mu", ct.c_double), ("thresh", ct.c_double),
                ("threshTr", ct.c_double), ("maxItr", ct.c_int32),
                ("basis", ct.c_int32)]


class Formations(ct.Structure):
    _fields_ = [("n", ct.c_int32), ("n_formations", ct.c_int32),
                ("p", ct.c_void_p), ("adj", ct.c_void_p), ("gains", ct.c_void_p),
                ("gain_off", ct.c_void_p), ("gain_planes", ct.c_int32),
                ("gains_tiled", ct.c_void_p)]


class SolveArgs(ct.Structure):
    _fields_ = [("B", ct.c_int32), ("fidx", ct.c_void_p), ("q", ct.c_void_p),
                ("vel", ct.c_void_p), ("P_in", ct.c_void_p), ("P_out", ct.c_void_p),
                ("status", ct.c_void_p), ("u", ct.c_void_p), ("u_safe", ct.c_void_p),
                ("ca_flag", ct.c_void_p), ("who", ct.c_void_p), ("workspace", ct.c_void_p),
                ("cntrl", CntrlGains), ("safety", SafetyParams),
                ("early_exit", ct.c_int32), ("do_control", ct.c_int32),
                ("align_Rt", ct.c_void_p), ("gate_margin", ct.c_void_p),
                ("skip_margin", ct.c_int32),
                ("P_rows", ct.c_void_p), ("P_rows_on", ct.c_void_p),
                ("ws_persistent", ct.c_int32)]


class ControlArgs(ct.Structure):
    """acl_control_args_t (DistCntrl + Safety for given assignments)."""
    _fields_ = [("B", ct.c_int32), ("fidx", ct.c_void_p), ("q", ct.c_void_p),
                ("vel", ct.c_void_p), ("P", ct.c_void_p), ("u", ct.c_void_p),
                ("u_safe", ct.c_void_p), ("ca_flag", ct.c_void_p), ("status", ct.c_void_p),
                ("workspace", ct.c_void_p), ("cntrl", CntrlGains), ("safety", SafetyParams),
                ("gate_margin", ct.c_void_p)]


class HungarianArgs(ct.Structure):
    """acl_hungarian_args_t (assignment.py:94-137, batched)."""
    _fields_ = [("B", ct.c_int32), ("fidx", ct.c_void_p), ("q", ct.c_void_p),
                ("P_last", ct.c_void_p), ("P_cmp", ct.c_void_p), ("P_opt", ct.c_void_p),
                ("cost", ct.c_void_p), ("align_Rt", ct.c_void_p), ("status", ct.c_void_p)]


class CbaaStepArgs(ct.Structure):
    """acl_cbaa_step_args_t (ABI 11): one CBAA bid iteration per vehicle
    (auctioneer.cpp:182-306,469-542)."""
    _fields_ = [("V", ct.c_int32), ("K", ct.c_int32)] + [(n, ct.c_void_p) for n in (
        "fidx", "vehid", "q", "Rt", "start", "price", "who", "cand_off", "cand_vehid",
        "cand_price", "cand_who", "task", "flags")]


class EpisodeParams(ct.Structure):
    """acl_episode_params_t (coordination.launch:6,24-25, safety.cpp:45-46,
    trial.sh:96, supervisor.py:47,61-62,121)."""
    _fields_ = [("control_dt", ct.c_double), ("auction_every", ct.c_int32),
                ("sample_every", ct.c_int32), ("bufflen", ct.c_int32),
                ("auction_latency", ct.c_int32), ("max_accel_xy", ct.c_double),
                ("max_accel_z", ct.c_double), ("bounds_min", ct.c_double * 3),
                ("bounds_max", ct.c_double * 3), ("orig_zero_vel_thr", ct.c_double),
                ("avg_active_ca_thr", ct.c_double), ("assignment", ct.c_int32)]


ASSIGN_CBAA = 0     # acl_episode_params_t::assignment (ABI 9)
ASSIGN_CENTRAL = 1


EPISODE_STATUS_DTYPE = np.dtype([("converged_step", "<i4"), ("gridlock_step", "<i4"),
                                 ("converged", "<i4"), ("gridlocked", "<i4"),
                                 ("n_auctions", "<u2"), ("n_invalid", "<u2"),
                                 ("n_skipped", "<u2"), ("n_disagree", "<u2"),
                                 ("n_samples", "<u4"), ("n_ca_steps", "<u4"),
                                 ("pending_step", "<i4"), ("n_restarted", "<u2"),
                                 ("per_vehicle", "<u2")])


class EpisodeArgs(ct.Structure):
    """acl_episode_args_t (closed-loop batched episodes)."""
    _fields_ = [("B", ct.c_int32), ("fidx", ct.c_void_p), ("q", ct.c_void_p),
                ("vel", ct.c_void_p), ("P", ct.c_void_p), ("flush", ct.c_void_p),
                ("est", ct.c_void_p), ("ring_u", ct.c_void_p), ("ring_ca", ct.c_void_p),
                ("step0", ct.c_int32), ("steps", ct.c_int32), ("q_hist", ct.c_void_p),
                ("vel_hist", ct.c_void_p), ("u_hist", ct.c_void_p), ("ca_hist", ct.c_void_p), ("P_hist", ct.c_void_p),
                ("workspace", ct.c_void_p), ("cntrl", CntrlGains), ("safety", SafetyParams),
                ("ep", EpisodeParams)]


class TrialParams(ct.Structure):
    """acl_trial_params_t (supervisor.py:47-62,88,121; coordination.launch:5)."""
    _fields_ = [("ep", EpisodeParams), ("tick_rate", ct.c_int32), ("settle_steps", ct.c_int32),
                ("hover_wait", ct.c_double), ("assignment_timeout", ct.c_double),
                ("formation_received_wait", ct.c_double), ("converged_wait", ct.c_double),
                ("gridlock_timeout", ct.c_double), ("trial_timeout", ct.c_double),
                ("alpha", ct.c_double)]


# supervisor.py State values (ACL_TRIAL_*)
TRIAL_HOVERING, TRIAL_WAITING, TRIAL_FLYING, TRIAL_IN_FORMATION = 3, 4, 5, 6
TRIAL_GRIDLOCK, TRIAL_COMPLETE, TRIAL_TERMINATE = 7, 8, 9

TRIAL_STATUS_DTYPE = np.dtype([(k, "<i4") for k in (
    "state", "last_state", "timer_ticks", "formation", "ticks", "received", "logging",
    "commit", "next_auction", "conv_len", "conv_head", "grid_len", "grid_head", "log_init",
    "t_start", "t_grid", "done_step")] + [("n_auctions", "<u2"), ("n_invalid", "<u2"),
                                          ("n_skipped", "<u2"), ("n_disagree", "<u2"),
                                          ("per_vehicle", "<i4")])


class TrialArgs(ct.Structure):
    """acl_trial_args_t (batched Monte-Carlo trials)."""
    _fields_ = [("B", ct.c_int32), ("K", ct.c_int32)] + [
        (k, ct.c_void_p) for k in ("fseq", "fidx", "q", "vel", "P", "flush", "ts", "ctl_on",
                                   "ring_u", "ring_ca", "posf", "dist", "t_conv", "t_avoid",
                                   "n_assign")] + [
        ("step0", ct.c_int32), ("steps", ct.c_int32)] + [
        (k, ct.c_void_p) for k in ("q_hist", "vel_hist", "u_hist", "ca_hist", "ctl_hist",
                                   "P_hist", "state_hist", "workspace")] + [
        ("cntrl", CntrlGains), ("safety", SafetyParams), ("tp", TrialParams)]


HUNG_BAD_INPUT = 0x01
HUNG_NONFINITE = 0x02
HUNG_CMP_INVALID = 0x04

_lib = None


def lib():
    """Load libaclswarm_amd.so; raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"aclswarm_amd: native library {LIB_PATH} is missing. Build it with "
            "`python -m aclswarm_amd.build` (hipcc --offload-arch=gfx950).")
    # torch before the library: torch bundles its own libamdhip64 under the
    # same SONAME, and whichever loads first is the process's HIP runtime;
    # loading torch first keeps it usable next to this library (the other
    # order leaves torch without a device)
    import torch  # noqa: F401
    L = ct.CDLL(LIB_PATH)
    VP, I32, I64, SZ = ct.c_void_p, ct.c_int32, ct.c_int64, ct.c_size_t
    L.acl_default_cntrl_gains.argtypes = [ct.POINTER(CntrlGains)]
    L.acl_default_safety_params.argtypes = [ct.POINTER(SafetyParams)]
    L.acl_default_admm_params.argtypes = [ct.POINTER(AdmmParams)]
    L.acl_formations_init.argtypes = [ct.POINTER(Formations), I32, I32]
    L.acl_formations_init.restype = None
    L.acl_max_vehicles.restype = I32
    L.acl_abi_version.restype = I32
    if L.acl_abi_version() != ABI_VERSION:
        raise RuntimeError(f"aclswarm_amd: {LIB_PATH} has ABI {L.acl_abi_version()}, this "
                           f"package expects {ABI_VERSION}: rebuild (python -m aclswarm_amd.build)")
    L.acl_solve_workspace_bytes.argtypes = [I32, I32]
    L.acl_solve_workspace_bytes.restype = ct.c_size_t
    L.acl_solve_batch.argtypes = [ct.POINTER(Formations), ct.POINTER(SolveArgs), VP]
    L.acl_solve_batch.restype = ct.c_int
    L.acl_count_edges.argtypes = [I32, VP]
    L.acl_count_edges.restype = I64
    L.acl_pack_adjacency.argtypes = [I32, VP, VP]
    L.acl_pack_adjacency.restype = ct.c_int
    L.acl_pack_gains.argtypes = [I32, VP, VP, VP]
    L.acl_pack_gains.restype = ct.c_int
    L.acl_gain_planes.argtypes = [I32, VP, VP]
    L.acl_gain_planes.restype = I32
    L.acl_pack_gains_planes.argtypes = [I32, VP, VP, I32, VP]
    L.acl_pack_gains_planes.restype = ct.c_int
    L.acl_tile_gains.argtypes = [ct.POINTER(Formations), VP, VP]
    L.acl_swarm_stats.argtypes = [VP, I32, VP, VP, VP]
    L.acl_swarm_stats.restype = I32
    L.acl_tile_gains.restype = ct.c_int
    L.acl_admm_solve_batch.argtypes = [I32, I32, VP, VP, VP, VP, ct.POINTER(AdmmParams), VP]
    L.acl_admm_solve_batch.restype = ct.c_int
    L.acl_control_batch.argtypes = [ct.POINTER(Formations), ct.POINTER(ControlArgs), VP]
    L.acl_control_batch.restype = ct.c_int
    L.acl_default_episode_params.argtypes = [ct.POINTER(EpisodeParams)]
    L.acl_default_episode_params.restype = None
    L.acl_episode_workspace_bytes.argtypes = [I32, I32]
    L.acl_episode_workspace_bytes.restype = SZ
    L.acl_episode_batch.argtypes = [ct.POINTER(Formations), ct.POINTER(EpisodeArgs), VP]
    L.acl_episode_batch.restype = ct.c_int
    L.acl_default_trial_params.argtypes = [ct.POINTER(TrialParams)]
    L.acl_default_trial_params.restype = None
    L.acl_trial_workspace_bytes.argtypes = [I32, I32]
    L.acl_trial_workspace_bytes.restype = SZ
    L.acl_trial_init.argtypes = [ct.POINTER(TrialArgs), I32, VP]
    L.acl_trial_init.restype = ct.c_int
    L.acl_trial_batch.argtypes = [ct.POINTER(Formations), ct.POINTER(TrialArgs), VP]
    L.acl_trial_batch.restype = ct.c_int
    L.acl_generate_formation_groups.argtypes = [I32, I32, VP, I32, ct.c_double, ct.c_double,
                                                ct.c_double, ct.c_double, I64, VP, VP, VP,
                                                VP, VP]
    L.acl_generate_formation_groups.restype = ct.c_int
    L.acl_hungarian_batch.argtypes = [ct.POINTER(Formations), ct.POINTER(HungarianArgs), VP]
    L.acl_hungarian_batch.restype = ct.c_int
    L.acl_cbaa_step_batch.argtypes = [ct.POINTER(Formations), ct.POINTER(CbaaStepArgs), VP]
    L.acl_cbaa_step_batch.restype = ct.c_int
    L.acl_write_assignment_log.argtypes = [ct.c_char_p, I32, VP, VP, VP, VP, VP, VP]
    L.acl_write_assignment_log.restype = ct.c_int
    L.acl_read_assignment_log.argtypes = [ct.c_char_p, ct.POINTER(I32), VP, VP, VP, VP, VP, VP]
    L.acl_read_assignment_log.restype = ct.c_int
    L.acl_device_count.restype = I32
    L.acl_set_device.argtypes = [I32]
    L.acl_set_device.restype = ct.c_int
    L.acl_malloc.argtypes = [ct.POINTER(VP), SZ]
    L.acl_malloc.restype = ct.c_int
    L.acl_free.argtypes = [VP]
    L.acl_free.restype = ct.c_int
    for fn in ("acl_memcpy_h2d", "acl_memcpy_d2h"):
        getattr(L, fn).argtypes = [VP, VP, SZ, VP]
        getattr(L, fn).restype = ct.c_int
    L.acl_memset.argtypes = [VP, ct.c_int, SZ, VP]
    L.acl_memset.restype = ct.c_int
    L.acl_stream_synchronize.argtypes = [VP]
    L.acl_stream_synchronize.restype = ct.c_int
    L.acl_last_error.restype = ct.c_char_p
    # diagnostics (not in the public header)
    L.acl_internal_kernel_timing.argtypes = [ct.c_int]
    L.acl_internal_kernel_timing.restype = None
    L.acl_internal_kernel_times.argtypes = [ct.POINTER(ct.c_double), ct.POINTER(ct.c_int)]
    L.acl_internal_kernel_times.restype = ct.c_int
    L.acl_internal_admm_flop_counter.argtypes = [VP]
    L.acl_internal_admm_flop_counter.restype = None
    if hasattr(L, "acl_internal_admm_mem_cap"):  # (absent from older experiment builds)
        L.acl_internal_admm_mem_cap.argtypes = [SZ]
        L.acl_internal_admm_mem_cap.restype = None
    L.acl_internal_psd_project.argtypes = [ct.c_int, ct.c_int, VP, ct.c_double, VP, ct.c_int,
                                           ct.POINTER(ct.c_int)]
    L.acl_internal_psd_project.restype = ct.c_int
    if hasattr(L, "acl_internal_price_sweep"):  # (absent from older experiment builds)
        L.acl_internal_price_sweep.argtypes = [VP, VP, VP, ct.c_int]
        L.acl_internal_price_sweep.restype = ct.c_int
    _lib = L
    return L


def check(rc, what="aclswarm_amd"):
    if rc != ACL_OK:
        msg = lib().acl_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def default_episode_params():
    e = EpisodeParams()
    lib().acl_default_episode_params(ct.byref(e))
    return e


def default_trial_params():
    t = TrialParams()
    lib().acl_default_trial_params(ct.byref(t))
    return t


def default_gains():
    g = CntrlGains()
    lib().acl_default_cntrl_gains(ct.byref(g))
    return g


def default_safety():
    s = SafetyParams()
    lib().acl_default_safety_params(ct.byref(s))
    return s


def default_admm_params():
    a = AdmmParams()
    lib().acl_default_admm_params(ct.byref(a))
    return a
