"""ctypes binding of libgymflock.so (include/gymflock.h).

No PyTorch here: the env talks to the HIP kernels through this thin C-ABI only.
The library is built in-tree (gym-flock_amd/lib/libgymflock.so, see
__graft_entry__.build()); if it is missing or no GPU is present, every call that
needs it raises — there is no CPU fallback in the product path.
"""
import ctypes
import math
import functools
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "GYMFLOCK_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libgymflock.so"))

GF_OK, GF_EINVAL, GF_EHIP, GF_ENOMEM, GF_ESTATE, GF_ECOMM = range(6)

FE_WITH_CONTROLLER = 0x01
FE_U_DEVICE = 0x02
FE_U_F64 = 0x04
FE_U_EXPERT = 0x08
FE_WITH_KNN = 0x10
FE_NO_NETWORK = 0x20
FE_NO_STATE_VALUES = 0x40
FE_U_RESIDENT = 0x80
FE_PACKED_NETWORK = 0x100
FE_OUT_MAPPED = 0x1  # fe_get_outputs flag


class FeConfig(ctypes.Structure):
    _fields_ = [("n_agents", ctypes.c_int32), ("n_envs", ctypes.c_int32),
                ("comm_radius", ctypes.c_double), ("dt", ctypes.c_double),
                ("action_scalar", ctypes.c_double), ("mean_pooling", ctypes.c_int32),
                ("centralized", ctypes.c_int32), ("n_neighbors", ctypes.c_int32),
                ("device", ctypes.c_int32)]


class FeBuffers(ctypes.Structure):
    _fields_ = [("x", ctypes.c_void_p), ("state_values", ctypes.c_void_p),
                ("network", ctypes.c_void_p), ("controls", ctypes.c_void_p),
                ("rewards", ctypes.c_void_p), ("knn_idx", ctypes.c_void_p),
                ("knn_obs", ctypes.c_void_p), ("stream", ctypes.c_void_p),
                ("adj_bits", ctypes.c_void_p), ("degree", ctypes.c_void_p)]


class FeVariant(ctypes.Structure):
    _fields_ = [("n_frozen", ctypes.c_int32), ("n_vel_zero", ctypes.c_int32),
                ("u_scale", ctypes.c_double), ("u_clip", ctypes.c_double),
                ("x_scale", ctypes.c_double), ("ctrl_clip", ctypes.c_double)]


class CovConfig(ctypes.Structure):
    _fields_ = [("n_robots", ctypes.c_int32), ("n_envs", ctypes.c_int32),
                ("max_nodes", ctypes.c_int32), ("episode_length", ctypes.c_int32),
                ("res", ctypes.c_double), ("motion_radius", ctypes.c_double),
                ("device", ctypes.c_int32), ("horizon", ctypes.c_int32)]


class CovMapConfig(ctypes.Structure):
    _fields_ = [("x_min", ctypes.c_double), ("x_max", ctypes.c_double), ("y_min", ctypes.c_double),
                ("y_max", ctypes.c_double), ("lattice_spacing", ctypes.c_double),
                ("world_radius", ctypes.c_double), ("road_radius", ctypes.c_double),
                ("near_radius", ctypes.c_double), ("link_radius", ctypes.c_double),
                ("n_cities", ctypes.c_int32)]


def map_config_default(motion_radius=5.5 * 1.2, xmax=120, ymax=120, n_cities=12, spacing=5.5):
    """The reference's map parameters (coverage.py:516-527): arena (-xmax, xmax, -ymax,
    ymax), lattice vectors of DELTA = 5.5, 12 cities U(-xmax, xmax)^2, roads and target
    links at motion_radius, lattice points within motion_radius / 1.4 of a road."""
    return CovMapConfig(-float(xmax), float(xmax), -float(ymax), float(ymax), float(spacing), float(xmax),
                        float(motion_radius), float(motion_radius) / 1.4, float(motion_radius), int(n_cities))


def map_lattice(mc=None):
    """generate_lattice's points (make_map.py:30-67) for a map configuration, computed by
    the library's host code (cov_map_lattice, no device needed): (n, 2) [y, x]."""
    mc = mc or map_config_default()
    lib = load()
    n = ctypes.c_int32(0)
    check(lib.cov_map_lattice(ctypes.byref(mc), None, ctypes.byref(n)))
    out = np.empty((n.value, 2), np.float64)
    check(lib.cov_map_lattice(ctypes.byref(mc), ptr(out), ctypes.byref(n)))
    return out


COV_MAP_SEED = 0x1
COV_MAP_CITIES = 0x2
COV_MAP_NEAR_DEGENERATE = 0x1
COV_MAP_TOO_MANY = 0x2
COV_MAP_TOO_FEW = 0x4
COV_MAP_OVERFLOW = 0x8

COV_ACTIONS_DEVICE = 0x1
COV_ACTIONS_RESIDENT = 0x2
COV_ACTIONS_GREEDY = 0x20
COV_OUT_DEVICE = 0x4
COV_FLAT_F32 = 0x8
COV_MASK_ALL = 0x10
COV_NEXT_GREEDY = 0x40
COV_GREEDY_RNG = 0x80


class GymFlockError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("libgymflock error %d: %s" % (code, msg))
        self.code = code


_P = ctypes.c_void_p
_I = ctypes.c_int
# name -> argtypes (every function returns int unless listed in _RESTYPE)
SIGNATURES = {
    "fe_create": [ctypes.POINTER(FeConfig), ctypes.POINTER(_P)],
    "fe_destroy": [_P],
    "fe_get_config": [_P, ctypes.POINTER(FeConfig)],
    "fe_set_params": [_P, ctypes.POINTER(FeConfig)],
    "fe_set_state": [_P, _P],
    "fe_set_state_env": [_P, _I, _P],
    "fe_get_state": [_P, _P],
    "fe_get_state_env": [_P, _I, _P],
    "fe_set_actions": [_P, _P, _I],
    "fe_compute_helpers": [_P, _I],
    "fe_step": [_P, _P, _I],
    "fe_step_host": [_P, _P, _P, _P, _P, _P, _I],
    "fe_step_host_knn": [_P, _P, _P, _P, _P, _P, _P, _I],
    "fe_step_host_knn_ctrl": [_P, _P, _P, _P, _P, _P, _P, _P, _I],
    "fe_controller": [_P, _I, _P],
    "fe_get_stats": [_P, _I, _P, _P],
    "fe_get_stats_ex": [_P, _I, _P, _P, _P],
    "fe_stats_summary": [_P, _P],
    "fe_get_state_values": [_P, _I, _P],
    "fe_get_network": [_P, _I, _P],
    "fe_get_network_rows": [_P, _I, _I, _I, _P],
    "fe_get_network_packed": [_P, _I, _P, _P],
    "fe_reset_synthetic": [_P, ctypes.c_uint64, ctypes.c_double],
    "fe_get_controls": [_P, _I, _P],
    "fe_get_rewards": [_P, _P],
    "fe_get_outputs": [_P, _I, _P, _P, _P, _I],
    "fe_host_alloc": [ctypes.c_size_t, ctypes.POINTER(_P)],
    "fe_host_free": [_P],
    "fe_get_knn": [_P, _I, _P, _P],
    "fe_device_buffers": [_P, ctypes.POINTER(FeBuffers)],
    "fe_sync": [_P],
    "fe_set_streams": [_P, _I],
    "fe_join": [_P],
    "fe_comm_unique_id": [_P],
    "fe_comm_init": [_P, _I, _I, _P],
    "fe_comm_init_timeout": [_P, _I, _I, _P, ctypes.c_double],
    "fe_check_shard_sizes": [_I, _P],
    "fe_comm_info": [_P, _P, _P, _P, ctypes.c_char_p, _I],
    "fe_comm_shard_sizes": [_P, _P, _P],
    "fe_allgather_rewards": [_P],
    "fe_get_gathered_rewards": [_P, _P],
    "fe_gathered_steps": [_P],
    "fe_allgather_stats": [_P],
    "fe_get_gathered_stats": [_P, _P],
    "fe_comm_destroy": [_P],
    "fe_debug_comm_gate": [_P, _I, ctypes.c_double],
    "fe_debug_comm_state": [_P, _P],
    "fe_runtime_info": [ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                        ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p, _I, ctypes.c_char_p, _I],
    "fe_set_variant": [_P, _P],
    "fe_set_dt": [_P, _P],
    "cov_create": [ctypes.POINTER(CovConfig), ctypes.POINTER(_P)],
    "cov_destroy": [_P],
    "cov_set_targets": [_P, _I, _I, _P],
    "cov_generate_maps": [_P, _P, _I, ctypes.c_uint64, _P, _I, _P, _P, _P],
    "cov_get_targets": [_P, _I, _P],
    "cov_map_lattice": [_P, _P, _P],
    "cov_reset": [_P, _P, _P],
    "cov_reset_seeded": [_P, ctypes.c_uint64, ctypes.c_double, _P, _P],
    "cov_step": [_P, _P, _I],
    "cov_step_expert": [_P, _I, _P, _P],
    "cov_set_actions": [_P, _P],
    "cov_set_rng": [_P, _P, _P],
    "cov_get_rng": [_P, _P, _P],
    "cov_step_host": [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I],
    "cov_set_robot_positions": [_P, _I, _P],
    "cov_get_obs": [_P, _I, _P, _P, _P, _P, _P],
    "cov_get_rewards": [_P, _P, _P],
    "cov_get_robots": [_P, _I, _P, _P],
    "cov_get_visited": [_P, _I, _P],
    "cov_get_n_motion": [_P, _P],
    "cov_sync": [_P],
    "cov_set_streams": [_P, _I],
    "cov_controller_greedy": [_P, _P, _P, _P],
    "cov_get_time_matrix": [_P, _I, _P, _P],
    "cov_get_actions": [_P, _P, _P],
    "cov_get_flat_obs": [_P, _P, _I],
    "cov_graphs_tuple_sizes": [_P, _P, _P, _I],
    "cov_get_graphs_tuple": [_P, _P, _P, _P, _P, _P, _P, _P, _I],
    "gu_create": [_I, ctypes.POINTER(_P)],
    "gu_destroy": [_P],
    "gu_radius_edges": [_P, _P, ctypes.c_int32, _P, ctypes.c_int32, ctypes.c_double, _I,
                        ctypes.POINTER(ctypes.c_int64)],
    "gu_k_edges": [_P, ctypes.c_int32, _P, ctypes.c_int32, _P, ctypes.c_int32, _I, _I,
                   ctypes.POINTER(ctypes.c_int64)],
    "gu_get_edges": [_P, _P, _P, _P, _P],
    "gu_nodes_within_radius": [_P, _P, ctypes.c_int32, _P, ctypes.c_int32, ctypes.c_double, _P],
    "fe_last_error": [],
    "fe_abi_version": [],
    "fe_diag": [_P, _I, _I, ctypes.POINTER(ctypes.c_double)],
    "fe_kernel_timing": [_P, _I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)],
    "cov_kernel_timing": [_P, _I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)],
}
_RESTYPE = {"fe_last_error": ctypes.c_char_p}

_lib = None


def load(path=None):
    """Load (once) and return the ctypes library; raises if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImportError("libgymflock.so not found at %s: build it with "
                          "`python -c 'import __graft_entry__ as g; g.build()'` "
                          "(or make -C gym-flock_amd/csrc)" % p)
    # RTLD_DEEPBIND: resolve the library's HIP/RCCL symbols against its own ROCm
    # dependencies even when another copy of the HIP runtime (e.g. PyTorch's bundled
    # one) is already in the process' global scope. GYMFLOCK_DEEPBIND=0 disables it.
    mode = ctypes.DEFAULT_MODE
    if os.environ.get("GYMFLOCK_DEEPBIND", "1") != "0":
        mode |= os.RTLD_DEEPBIND
    lib = ctypes.CDLL(p, mode=mode)
    for name, args in SIGNATURES.items():
        if not hasattr(lib, name) and os.environ.get("GYMFLOCK_LIB"):
            continue  # an older library selected for an A/B run lacks newer entry points
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPE.get(name, ctypes.c_int)
    if path is None:
        _lib = lib
    return lib


def check(rc):
    if rc != GF_OK:
        raise GymFlockError(rc, load().fe_last_error().decode(errors="replace"))


class HostPool:
    """Page-locked host buffers (fe_host_alloc) handed out as fresh numpy arrays.

    The drop-in env returns new arrays every step (the reference's step() does, and
    callers may keep them). Copying the step's outputs into page-locked memory runs at
    full link rate and touches no fresh pageable pages; each array here owns its buffer
    until the array (and every view of it) is released, then the buffer returns to the
    pool for the next step. Page-locked bytes held by live arrays are capped: past the
    cap (a caller keeping many steps' outputs), arrays are ordinary numpy memory."""

    def __init__(self, cap_bytes=256 << 20):
        import collections
        import threading
        self.cap = int(cap_bytes)
        self._live = 0  # page-locked bytes handed out and not yet reclaimed
        self.free = {}
        self.lock = threading.Lock()
        # buffers handed out, oldest first, as (weak reference to the ctypes buffer every
        # array and view of it keeps alive, address, bytes). A buffer is reclaimed once its
        # reference is dead; each allocation looks at a few of the oldest entries (a step's
        # arrays are usually released within a step or two). No finalizer callbacks: they
        # cost more than the step's own launch overhead and can fire inside any allocation.
        self.out = collections.deque()

    def _reclaim(self, budget):
        # caller holds self.lock; checks at most `budget` of the oldest entries (all: -1)
        n = len(self.out) if budget < 0 else min(budget, len(self.out))
        for _ in range(n):
            ref, p, nbytes = self.out.popleft()
            if ref() is None:
                self._live -= nbytes
                self.free.setdefault(nbytes, []).append(p)
            else:
                self.out.append((ref, p, nbytes))

    @property
    def live(self):
        """Page-locked bytes held by live arrays (every released one reclaimed first)."""
        with self.lock:
            self._reclaim(-1)
            return self._live

    def array(self, shape, dtype):
        return self.array_addr(shape, dtype)[0]

    def array_addr(self, shape, dtype):
        """(array, its address): a page-locked array from the pool, or past the cap (or if
        page-locked memory runs out) an ordinary numpy array and None."""
        dtype = np.dtype(dtype)
        nbytes = math.prod(shape) * dtype.itemsize
        if nbytes == 0:
            return np.empty(shape, dtype), None
        buf, p = self.block_addr(nbytes)
        if p is None:
            return np.empty(shape, dtype), None
        return np.frombuffer(buf, dtype=dtype).reshape(shape), p

    def block_addr(self, nbytes):
        """(ctypes byte buffer, its address) of `nbytes` page-locked bytes from the pool, or
        (None, None) past the cap or when page-locked memory runs out. Arrays made over the
        buffer (np.ndarray(buffer=...)) keep it alive; it returns to the pool once all of
        them are released."""
        import weakref
        with self.lock:
            self._reclaim(4)
            lst = self.free.get(nbytes)
            if not lst:
                self._reclaim(-1)
                lst = self.free.get(nbytes)
            p = lst.pop() if lst else None
            if p is None and self._live + nbytes > self.cap:
                return None, None
            self._live += nbytes
        if p is None:
            out = ctypes.c_void_p()
            try:
                check(load().fe_host_alloc(nbytes, ctypes.byref(out)))
            except GymFlockError:
                with self.lock:
                    self._live -= nbytes
                return None, None
            p = out.value
        buf = (ctypes.c_uint8 * nbytes).from_address(p)
        with self.lock:
            self.out.append((weakref.ref(buf), p, nbytes))
        return buf, p

    def trim(self):
        """Free the recycled (unused) buffers."""
        with self.lock:
            self._reclaim(-1)
            ps = [p for lst in self.free.values() for p in lst]
            self.free = {}
        for p in ps:
            load().fe_host_free(ctypes.c_void_p(p))


_host_pool = None


def host_pool():
    """The process-wide HostPool of the drop-in envs."""
    global _host_pool
    if _host_pool is None:
        _host_pool = HostPool()
    return _host_pool


class PinnedArray:
    """A page-locked host array owned by one object (fe_host_alloc / fe_host_free), e.g.
    the drop-in env's action buffer, which the step kernel reads in place."""

    def __init__(self, shape, dtype):
        dtype = np.dtype(dtype)
        nbytes = max(1, int(np.prod(shape)) * dtype.itemsize)
        out = ctypes.c_void_p()
        check(load().fe_host_alloc(nbytes, ctypes.byref(out)))
        self.addr = out.value
        self.a = np.frombuffer((ctypes.c_uint8 * nbytes).from_address(self.addr), dtype=dtype,
                               count=int(np.prod(shape))).reshape(shape)

    def close(self):
        if getattr(self, "addr", None):
            self.a = None
            load().fe_host_free(ctypes.c_void_p(self.addr))
            self.addr = None

    __del__ = close


def u_is_f64(u):
    """Whether the reference's `u * action_scalar` (flocking_relative.py:95) computes in
    float64 for this action array (NumPy's promotion: float32 stays float32, float64 and
    integer arrays go to float64).

    float16 actions are the exception: NumPy keeps `u * 10.0 * dt * dt * 0.5` in float16
    (legacy value-based casting and NEP 50 alike), while the kernels have float32 and
    float64 arithmetic only. They are cast to float32 and computed exactly as float32
    actions of the same values are (tests/test_flock_gpu.py pins that); parity with the
    reference's float16 rounding is unpinned."""
    d = u.dtype
    if d == np.float32 or d == np.float16:
        return False
    return d == np.float64 or np.result_type(d, 10.0) != np.float32


def runtime_info():
    """The HIP runtime and RCCL libgymflock is bound to in this process (fe_runtime_info):
    {hip_runtime, hip_driver, rccl: versions; hip_lib, rccl_lib: shared-object paths}."""
    rt, dv, rc = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    hp, rp = ctypes.create_string_buffer(512), ctypes.create_string_buffer(512)
    check(load().fe_runtime_info(ctypes.byref(rt), ctypes.byref(dv), ctypes.byref(rc), hp, 512, rp, 512))
    return {"hip_runtime": rt.value, "hip_driver": dv.value, "rccl": rc.value,
            "hip_lib": hp.value.decode(errors="replace"), "rccl_lib": rp.value.decode(errors="replace")}


def check_shard_sizes(n_envs):
    """fe_comm_init's shard-size rule on a list of per-rank env counts (host only)."""
    a = np.ascontiguousarray(n_envs, dtype=np.int32)
    check(load().fe_check_shard_sizes(len(a), a.ctypes.data_as(ctypes.c_void_p)))


def ptr(a):
    """Pointer to a C-contiguous numpy array (None passes NULL)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return a.ctypes.data_as(ctypes.c_void_p)


class FlockHandle:
    """Owns one fe_handle: B envs x N agents of FlockingRelative on one GPU."""

    def __init__(self, n_agents, n_envs=1, comm_radius=0.9, dt=0.01, action_scalar=10.0,
                 mean_pooling=True, centralized=True, n_neighbors=0, device=0):
        self.lib = load()
        self.cfg = FeConfig(int(n_agents), int(n_envs), float(comm_radius), float(dt),
                            float(action_scalar), int(bool(mean_pooling)), int(bool(centralized)),
                            int(n_neighbors), int(device))
        self.n_agents, self.n_envs, self.n_neighbors = int(n_agents), int(n_envs), int(n_neighbors)
        h = ctypes.c_void_p()
        check(self.lib.fe_create(ctypes.byref(self.cfg), ctypes.byref(h)))
        self.h = h

    def close(self):
        h = getattr(self, "h", None)
        if h:
            self.lib.fe_destroy(h)
            h.value = None  # any copy of the handle object now passes NULL (GF_EINVAL)
            self.h = None

    __del__ = close

    def set_params(self, comm_radius, dt, action_scalar, mean_pooling, centralized):
        """New comm_radius / dt / action_scalar / mean_pooling / centralized for the later
        launches, the state kept (fe_set_params)."""
        c = FeConfig(self.cfg.n_agents, self.cfg.n_envs, float(comm_radius), float(dt), float(action_scalar),
                     int(bool(mean_pooling)), int(bool(centralized)), self.cfg.n_neighbors, self.cfg.device)
        check(self.lib.fe_set_params(self.h, ctypes.byref(c)))
        self.cfg = c

    # -- variants (include/gymflock.h fe_variant)
    def set_variant(self, n_frozen=0, n_vel_zero=0, u_scale=None, u_clip=0.0, x_scale=1.0,
                    ctrl_clip=0.0):
        """Select a flocking variant for later steps; no arguments = FlockingRelative."""
        v = FeVariant(int(n_frozen), int(n_vel_zero),
                      float(self.cfg.action_scalar if u_scale is None else u_scale),
                      float(u_clip or 0.0), float(x_scale), float(ctrl_clip or 0.0))
        check(self.lib.fe_set_variant(self.h, ctypes.byref(v)))

    def clear_variant(self):
        check(self.lib.fe_set_variant(self.h, None))

    def set_dt(self, dt):
        """Per-env dt (B,) for the following steps; None reverts to the config dt."""
        if dt is None:
            check(self.lib.fe_set_dt(self.h, None))
            return
        d = np.ascontiguousarray(np.broadcast_to(np.asarray(dt, np.float64), (self.n_envs,)))
        check(self.lib.fe_set_dt(self.h, ptr(d)))

    # -- state
    def reset_synthetic(self, seed=0, v_max=5.0):
        """Synthetic init of every env in the library (fe_reset_synthetic)."""
        check(self.lib.fe_reset_synthetic(self.h, int(seed), float(v_max)))

    def set_state(self, x, env=None):
        x = np.ascontiguousarray(x, dtype=np.float64)
        if env is None:
            assert x.shape == (self.n_envs, self.n_agents, 4), x.shape
            check(self.lib.fe_set_state(self.h, ptr(x)))
        else:
            assert x.shape == (self.n_agents, 4), x.shape
            check(self.lib.fe_set_state_env(self.h, int(env), ptr(x)))

    def get_state(self, env=None):
        if env is None:
            x = np.empty((self.n_envs, self.n_agents, 4))
            check(self.lib.fe_get_state(self.h, ptr(x)))
        else:
            x = np.empty((self.n_agents, 4))
            check(self.lib.fe_get_state_env(self.h, int(env), ptr(x)))
        return x

    # -- hot path
    def compute_helpers(self, flags=0):
        check(self.lib.fe_compute_helpers(self.h, int(flags)))

    def set_actions(self, u):
        """Upload (B,N,2) actions to the resident buffer used by FE_U_RESIDENT."""
        u = np.asarray(u)
        f64 = u_is_f64(u)
        u = np.ascontiguousarray(u, dtype=np.float64 if f64 else np.float32)
        assert u.shape == (self.n_envs, self.n_agents, 2), u.shape
        check(self.lib.fe_set_actions(self.h, ptr(u), int(f64)))

    def step(self, u=None, flags=0):
        """u: host ndarray (B,N,2) (float32 arithmetic for float32/float16 actions, else
        float64, as NumPy promotes u * 10.0), or a device pointer (int) with FE_U_DEVICE,
        or None with FE_U_EXPERT / FE_U_RESIDENT."""
        if flags & (FE_U_EXPERT | FE_U_RESIDENT):
            check(self.lib.fe_step(self.h, None, int(flags)))
        elif flags & FE_U_DEVICE:
            check(self.lib.fe_step(self.h, ctypes.c_void_p(int(u)), int(flags)))
        else:
            u = np.asarray(u)
            if u_is_f64(u):
                flags |= FE_U_F64
                u = u.astype(np.float64, copy=False)
            else:
                u = u.astype(np.float32, copy=False)
                flags &= ~FE_U_F64
            u = np.ascontiguousarray(u)
            assert u.shape == (self.n_envs, self.n_agents, 2), u.shape
            check(self.lib.fe_step(self.h, ptr(u), int(flags)))

    def step_host(self, u_addr, f64, sv, net, rew, ctrl):
        """fe_step_host: one launch and one wait. u_addr: address of (B,N,2) host actions
        (page-locked ones are read in place) or None (compute_helpers); sv / net / rew /
        ctrl: addresses of host destinations or None (page-locked ones are written by the
        kernel directly). Addresses are ints (the drop-in env passes pool addresses)."""
        rc = self.lib.fe_step_host(self.h, u_addr, sv, net, rew, ctrl, FE_U_F64 if f64 else 0)
        if rc:
            check(rc)

    def step_host_knn(self, u_addr, f64, sv, net, rew, idx, obs, ctrl=None):
        """fe_step_host_knn(_ctrl): step_host plus the new state's k nearest (addresses of
        host destinations, page-locked ones written in place; any may be None but not both
        idx and obs), and with ctrl the expert action of the new state (fused)."""
        if ctrl is None:
            rc = self.lib.fe_step_host_knn(self.h, u_addr, sv, net, rew, idx, obs, FE_U_F64 if f64 else 0)
        else:
            rc = self.lib.fe_step_host_knn_ctrl(self.h, u_addr, sv, net, rew, ctrl, idx, obs,
                                                FE_U_F64 if f64 else 0)
        if rc:
            check(rc)

    def controller(self, centralized=None):
        out = np.empty((self.n_envs, self.n_agents, 2))
        c = -1 if centralized is None else int(bool(centralized))
        check(self.lib.fe_controller(self.h, c, ptr(out)))
        return out

    def stats(self, env=0):
        """(vel_diffs, min_dists, degree) of one env's current state."""
        vd = np.empty(self.n_agents)
        md = np.empty(self.n_agents)
        deg = np.empty(self.n_agents, np.int32)
        check(self.lib.fe_get_stats_ex(self.h, int(env), ptr(vd), ptr(md), ptr(deg)))
        return vd, md, deg

    def stats_summary(self):
        """(B, 2): np.mean(vel_diffs), np.mean(min_dists) of every env's current state."""
        out = np.empty((self.n_envs, 2))
        check(self.lib.fe_stats_summary(self.h, ptr(out)))
        return out

    # -- outputs
    def state_values(self, env=None):
        shape = (self.n_envs, self.n_agents, 6) if env is None else (self.n_agents, 6)
        out = np.empty(shape, np.float32)
        check(self.lib.fe_get_state_values(self.h, -1 if env is None else int(env), ptr(out)))
        return out

    def network(self, env=None):
        n = self.n_agents
        shape = (self.n_envs, n, n) if env is None else (n, n)
        out = np.empty(shape, np.float32)
        check(self.lib.fe_get_network(self.h, -1 if env is None else int(env), ptr(out)))
        return out

    def network_rows(self, env, row0, nrows):
        out = np.empty((nrows, self.n_agents), np.float32)
        check(self.lib.fe_get_network_rows(self.h, int(env), int(row0), int(nrows), ptr(out)))
        return out

    def network_packed(self, env=None):
        """(bits uint64 [(B,)N,ceil(N/64)], degree int32 [(B,)N]) of the last
        FE_PACKED_NETWORK step; adj(i,j) = bits[i, j//64] >> (j%64) & 1."""
        wn = (self.n_agents + 63) // 64
        lead = (self.n_envs,) if env is None else ()
        bits = np.empty(lead + (self.n_agents, wn), np.uint64)
        deg = np.empty(lead + (self.n_agents,), np.int32)
        check(self.lib.fe_get_network_packed(self.h, -1 if env is None else int(env), ptr(bits), ptr(deg)))
        return bits, deg

    def controls(self, env=None):
        shape = (self.n_envs, self.n_agents, 2) if env is None else (self.n_agents, 2)
        out = np.empty(shape)
        check(self.lib.fe_get_controls(self.h, -1 if env is None else int(env), ptr(out)))
        return out

    def rewards(self):
        out = np.empty(self.n_envs)
        check(self.lib.fe_get_rewards(self.h, ptr(out)))
        return out

    def outputs(self, env=None, pool=None):
        """(state_values, network, rewards) in one call and one stream sync
        (fe_get_outputs). With a HostPool the arrays are page-locked buffers from it
        (fresh arrays to the caller, recycled once released)."""
        n = self.n_agents
        lead = (self.n_envs, n) if env is None else (n,)
        new = pool.array if pool is not None else np.empty
        sv = new(lead + (6,), np.float32)
        net = new(lead + (n,), np.float32)
        rw = np.empty(self.n_envs)
        if pool is not None:
            rw = pool.array((self.n_envs,), np.float64)
        # pool arrays are page-locked (those past the pool's cap are not: the library
        # copies those by DMA), written by one copy kernel (FE_OUT_MAPPED)
        check(self.lib.fe_get_outputs(self.h, -1 if env is None else int(env), ptr(sv), ptr(net), ptr(rw),
                                      FE_OUT_MAPPED if pool is not None else 0))
        return sv, net, rw

    def knn(self, env=None):
        k, n = self.n_neighbors, self.n_agents
        lead = (self.n_envs, n) if env is None else (n,)
        idx = np.empty(lead + (k,), np.int32)
        obs = np.empty(lead + (4 * k,), np.float32)
        check(self.lib.fe_get_knn(self.h, -1 if env is None else int(env), ptr(idx), ptr(obs)))
        return idx, obs

    def device_buffers(self):
        b = FeBuffers()
        check(self.lib.fe_device_buffers(self.h, ctypes.byref(b)))
        return b

    def sync(self):
        check(self.lib.fe_sync(self.h))

    # -- timing (bench)
    def set_streams(self, n):
        """Launches per step: 2 (default) splits the env batch over two HIP streams so
        consecutive launches overlap; 1 keeps every step on the handle's stream."""
        check(self.lib.fe_set_streams(self.h, int(n)))

    def join(self):
        """Order the handle's stream after all outstanding work (no host wait)."""
        check(self.lib.fe_join(self.h))

    def timing_start(self, every=1):
        """Time every `every`-th step launch with HIP events (fe_kernel_timing); with
        split steps, the device time per step of the whole window instead."""
        check(self.lib.fe_kernel_timing(self.h, int(every), None, None))

    def timing_stop(self):
        ms, n = ctypes.c_double(), ctypes.c_int64()
        check(self.lib.fe_kernel_timing(self.h, 0, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def diag_fill(self, nontemporal=False, reps=10):
        ms = ctypes.c_double()
        check(self.lib.fe_diag(self.h, 1 if nontemporal else 0, int(reps), ctypes.byref(ms)))
        return ms.value

    def diag_switches(self, bits):
        check(self.lib.fe_diag(self.h, 0x10000 | int(bits), 1, None))

    # -- RCCL metrics path
    @staticmethod
    def comm_unique_id():
        buf = (ctypes.c_uint8 * 128)()
        check(load().fe_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
        return bytes(buf)

    def comm_init(self, nranks, rank, uid, timeout=300.0):
        """RCCL communicator for the metrics all-gathers, bounded by `timeout` seconds
        (also the bound of every later wait for a collective). Shards may differ in size."""
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(self.lib.fe_comm_init_timeout(self.h, int(nranks), int(rank), ctypes.cast(buf, ctypes.c_void_p),
                                            float(timeout)))
        self.nranks = int(nranks)
        self.shard_sizes, self.max_envs = self.comm_shard_sizes()

    def comm_shard_sizes(self):
        """(every rank's n_envs as a list, the largest: the gathers' padded width)."""
        sizes = np.empty(self.nranks, np.int32)
        mx = ctypes.c_int32()
        check(self.lib.fe_comm_shard_sizes(self.h, ptr(sizes), ctypes.byref(mx)))
        return [int(v) for v in sizes], int(mx.value)

    def comm_info(self):
        """The communicator as RCCL reports it: {count, user_rank, device, pci_bus_id}."""
        c, r, d = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        bus = ctypes.create_string_buffer(64)
        check(self.lib.fe_comm_info(self.h, ctypes.byref(c), ctypes.byref(r), ctypes.byref(d), bus, 64))
        return {"count": c.value, "user_rank": r.value, "device": d.value,
                "pci_bus_id": bus.value.decode(errors="replace")}

    def comm_destroy(self):
        check(self.lib.fe_comm_destroy(self.h))

    def debug_comm_gate(self, close, max_seconds=30.0):
        """Tests only: hold (close=True) or release the collectives' side stream with a
        bounded spin kernel, as a collective stuck on a dead peer would (fe_debug_comm_gate)."""
        check(self.lib.fe_debug_comm_gate(self.h, int(bool(close)), float(max_seconds)))

    _COMM_STATE = ("reuse_checks", "reuse_copy_done", "reuse_wait_rc", "reuse_async_state", "listed_after_gather",
                   "gather_copy_done", "gate_stream_query", "wait_polls", "gate_started", "gate_ended",
                   "comm_live", "listed_now")

    def debug_comm_state(self):
        """Tests only: what the metrics path saw (fe_debug_comm_state) as a dict."""
        out = np.zeros(12, np.int32)
        check(self.lib.fe_debug_comm_state(self.h, ptr(out)))
        return dict(zip(self._COMM_STATE, (int(v) for v in out)))

    def allgather_rewards(self):
        """Enqueue the all-gather of every step's rewards since the previous one."""
        check(self.lib.fe_allgather_rewards(self.h))

    def gathered_rewards(self):
        """(nranks, steps, max_envs) rewards of the steps covered by the latest all-gather
        (rank r's columns past its n_envs are zero padding)."""
        steps = self.lib.fe_gathered_steps(self.h)
        out = np.empty((self.nranks, max(steps, 1), self.max_envs))
        check(self.lib.fe_get_gathered_rewards(self.h, ptr(out)))
        return out[:, :steps]

    def allgather_stats(self):
        """Enqueue the all-gather of every rank's stats_summary() (side stream)."""
        check(self.lib.fe_allgather_stats(self.h))

    def gathered_stats(self):
        """(nranks, max_envs, 2) summaries of the latest stats all-gather, rank-major."""
        out = np.empty((self.nranks, self.max_envs, 2))
        check(self.lib.fe_get_gathered_stats(self.h, ptr(out)))
        return out


class CoverageHandle:
    """Owns one cov_handle: B Coverage-v0 envs with R robots, max_nodes padded nodes."""

    def __init__(self, n_robots, n_envs=1, max_nodes=500, episode_length=75, res=5.5,
                 motion_radius=None, device=0, horizon=10):
        self.lib = load()
        if motion_radius is None:
            motion_radius = res * 1.2
        self.cfg = CovConfig(int(n_robots), int(n_envs), int(max_nodes), int(episode_length),
                             float(res), float(motion_radius), int(device), int(horizon))
        self.n_robots, self.n_envs, self.max_nodes = int(n_robots), int(n_envs), int(max_nodes)
        self.t_max = self.max_nodes - self.n_robots
        h = ctypes.c_void_p()
        check(self.lib.cov_create(ctypes.byref(self.cfg), ctypes.byref(h)))
        self.h = h
        # the resident-action and fused greedy steps with their arguments bound: a step is
        # ~7 us, host-bound
        self._step_resident = functools.partial(self.lib.cov_step, h, None, COV_ACTIONS_RESIDENT)
        self._step_greedy = functools.partial(self.lib.cov_step, h, None, COV_ACTIONS_GREEDY)
        self._step_greedy_rng = functools.partial(self.lib.cov_step, h, None, COV_ACTIONS_GREEDY | COV_GREEDY_RNG)

    def close(self):
        h = getattr(self, "h", None)
        if h:
            self.lib.cov_destroy(h)
            # the bound resident-step partial holds this same object: it now passes NULL
            # (GF_EINVAL) instead of the freed handle
            h.value = None
            self.h = None

    __del__ = close

    def timing_start(self, every=1):
        """Time every `every`-th step launch with HIP events (cov_kernel_timing)."""
        check(self.lib.cov_kernel_timing(self.h, int(every), None, None))

    def timing_stop(self):
        ms, n = ctypes.c_double(), ctypes.c_int64()
        check(self.lib.cov_kernel_timing(self.h, 0, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def set_targets(self, targets, env=-1):
        t = np.ascontiguousarray(targets, dtype=np.float64)
        assert t.ndim == 2 and t.shape[1] == 2, t.shape
        check(self.lib.cov_set_targets(self.h, int(env), int(t.shape[0]), ptr(t)))

    def generate_maps(self, map_seed=None, cities=None, env=-1, map_config=None, fetch=True):
        """New target maps on the device (cov_generate_maps, coverage.py:516-527) for env
        `env` (-1: every env), then their motion graphs. cities=None: drawn from each env's
        map stream, seeded np.random.seed(map_seed + b) when map_seed is given, else
        continued from the previous maps; cities (n_sel, n_cities, 2): given. Returns
        (n_targets, status, cities) per selected env (None with fetch=False)."""
        mc = map_config or map_config_default(self.cfg.motion_radius)
        nsel = self.n_envs if env < 0 else 1
        flags = 0
        c = None
        if cities is not None:
            c = np.ascontiguousarray(cities, dtype=np.float64).reshape(nsel, mc.n_cities, 2)
            flags |= COV_MAP_CITIES
        elif map_seed is not None:
            flags |= COV_MAP_SEED
        n = np.full(nsel, -1, np.int32) if fetch else None
        st = np.zeros(nsel, np.int32) if fetch else None
        co = np.empty((nsel, mc.n_cities, 2), np.float64) if fetch else None
        rc = self.lib.cov_generate_maps(self.h, ctypes.byref(mc), int(env), int(map_seed or 0), ptr(c), flags,
                                        ptr(n), ptr(st), ptr(co))
        if rc:
            err = GymFlockError(rc, self.lib.fe_last_error().decode(errors="replace"))
            err.n_targets, err.status = n, st  # which envs' maps were refused, and why
            raise err
        return (n, st, co) if fetch else None

    def targets(self, env, n_targets):
        """The (n_targets, 2) targets of env `env`'s current map (n_targets: its size, as
        generate_maps returned it)."""
        out = np.empty((int(n_targets), 2), np.float64)
        check(self.lib.cov_get_targets(self.h, int(env), ptr(out)))
        return out

    def reset(self, start, visited):
        """start: (B,R) target-local start nodes; visited: (B, max_nodes-R) 0/1."""
        st = np.ascontiguousarray(start, dtype=np.int32)
        vi = np.ascontiguousarray(visited, dtype=np.uint8)
        assert st.shape == (self.n_envs, self.n_robots), st.shape
        assert vi.shape == (self.n_envs, self.t_max), vi.shape
        check(self.lib.cov_reset(self.h, ptr(st), ptr(vi)))

    def reset_seeded(self, seed, frac_active=0.5, fetch=True):
        """reset() with its random draws on the device (cov_reset_seeded): env b draws from
        RandomState(seed + b) as the reference's reset does; the streams stay on the device
        for the greedy expert's fallback draws. Returns (start (B,R), visited (B,t_max)) or,
        with fetch=False, None."""
        st = np.empty((self.n_envs, self.n_robots), np.int32) if fetch else None
        vi = np.empty((self.n_envs, self.t_max), np.uint8) if fetch else None
        check(self.lib.cov_reset_seeded(self.h, int(seed), float(frac_active), ptr(st) if fetch else None,
                                        ptr(vi) if fetch else None))
        return (st, vi) if fetch else None

    def step(self, actions=None, resident=False, greedy=False, rng=False):
        """actions (B,R) host ints; or resident=True (the last set/greedy actions); or
        greedy=True: controller(greedy=True)'s actions computed inside the step's launch
        (fallback robots take action 0, needs_random flags them; with rng=True they draw
        np_random.choice(4) from the envs' device streams, set_rng)."""
        if resident or greedy:
            rc = (self._step_greedy_rng() if rng else self._step_greedy()) if greedy else self._step_resident()
            if rc:
                check(rc)
            return
        a = np.ascontiguousarray(np.asarray(actions).reshape(self.n_envs, self.n_robots), dtype=np.int32)
        check(self.lib.cov_step(self.h, ptr(a), 0))

    def step_expert(self, n_steps, fetch=True):
        """n_steps fused greedy expert steps with the device fallback draws in one launch
        (cov_step_expert): the same as n_steps step(greedy=True, rng=True) calls. Returns
        every step's (rewards (n_steps,B), done (n_steps,B) bool), or None with fetch=False
        (asynchronous)."""
        r = np.empty((int(n_steps), self.n_envs)) if fetch else None
        d = np.empty((int(n_steps), self.n_envs), np.uint8) if fetch else None
        check(self.lib.cov_step_expert(self.h, int(n_steps), ptr(r) if fetch else None, ptr(d) if fetch else None))
        return (r, d.astype(bool)) if fetch else None

    def set_actions(self, actions):
        a = np.ascontiguousarray(np.asarray(actions).reshape(self.n_envs, self.n_robots), dtype=np.int32)
        check(self.lib.cov_set_actions(self.h, ptr(a)))

    def set_rng(self, states):
        """Every env's np_random stream for step(greedy=True, rng=True): a list of B
        RandomState objects (or get_state() tuples), copied to the device (cov_set_rng)."""
        keys = np.empty((self.n_envs, 624), np.uint32)
        pos = np.empty(self.n_envs, np.int32)
        assert len(states) == self.n_envs
        for b, st in enumerate(states):
            st = st.get_state() if hasattr(st, "get_state") else st
            assert st[0] == "MT19937" and len(st[1]) == 624, "a legacy RandomState (MT19937) state"
            keys[b], pos[b] = st[1], st[2]
        check(self.lib.cov_set_rng(self.h, ptr(keys), ptr(pos)))

    def get_rng(self):
        """(keys (B,624) uint32, pos (B) int32): the device streams after the steps that drew
        from them; RandomState.set_state(("MT19937", keys[b], pos[b])) continues env b's."""
        keys = np.empty((self.n_envs, 624), np.uint32)
        pos = np.empty(self.n_envs, np.int32)
        check(self.lib.cov_get_rng(self.h, ptr(keys), ptr(pos)))
        return keys, pos

    def step_host(self, actions, nodes, edges, senders, receivers, step, reward, done, closest,
                  next_actions=None, needs_random=None):
        """cov_step_host: one launch and one wait; the arguments after `actions` (B,R) int32
        are addresses (ints) of host destinations or None, page-locked ones written by the
        kernel in place. With next_actions / needs_random, controller(greedy=True)'s actions
        of the resulting state come back too (COV_NEXT_GREEDY)."""
        flags = COV_NEXT_GREEDY if (next_actions is not None or needs_random is not None) else 0
        rc = self.lib.cov_step_host(self.h, actions.ctypes.data, nodes, edges, senders, receivers, step, reward,
                                    done, closest, next_actions, needs_random, flags)
        if rc:
            check(rc)

    def actions(self):
        """(resident actions (B,R) int32, needs_random (B,R) bool) of the last greedy call or
        set_actions."""
        a = np.empty((self.n_envs, self.n_robots), np.int32)
        r = np.empty((self.n_envs, self.n_robots), np.uint8)
        check(self.lib.cov_get_actions(self.h, ptr(a), ptr(r)))
        return a, r.astype(bool)

    def set_robot_positions(self, env, xr):
        x = np.ascontiguousarray(xr, dtype=np.float64)
        assert x.shape == (self.n_robots, 2)
        check(self.lib.cov_set_robot_positions(self.h, int(env), ptr(x)))

    def obs(self, env=0):
        m = self.max_nodes
        nodes = np.empty((m, 3), np.float32)
        edges = np.empty((4 * m, 1), np.float32)
        snd = np.empty(4 * m, np.int32)
        rcv = np.empty(4 * m, np.int32)
        step = np.empty((1, 1), np.int64)
        check(self.lib.cov_get_obs(self.h, int(env), ptr(nodes), ptr(edges), ptr(snd), ptr(rcv), ptr(step)))
        return {"nodes": nodes, "edges": edges, "senders": snd, "receivers": rcv, "step": step}

    def motion_edges(self, env=0, n=None):
        """The first n (default: the env's motion-edge count) senders and receivers of env's
        observation, i.e. its motion graph (global node indices), without the rest."""
        m = self.max_nodes
        snd = np.empty(4 * m, np.int32)
        rcv = np.empty(4 * m, np.int32)
        check(self.lib.cov_get_obs(self.h, int(env), None, None, ptr(snd), ptr(rcv), None))
        n = int(self.n_motion()[env]) if n is None else int(n)
        return snd[:n], rcv[:n]

    def rewards(self):
        r = np.empty(self.n_envs)
        d = np.empty(self.n_envs, np.uint8)
        check(self.lib.cov_get_rewards(self.h, ptr(r), ptr(d)))
        return r, d.astype(bool)

    def robots(self, env=0):
        x = np.empty((self.n_robots, 2))
        n = np.empty(self.n_robots, np.int32)
        check(self.lib.cov_get_robots(self.h, int(env), ptr(x), ptr(n)))
        return x, n

    def visited(self, env=0):
        v = np.empty(self.t_max, np.uint8)
        check(self.lib.cov_get_visited(self.h, int(env), ptr(v)))
        return v

    def n_motion(self):
        n = np.empty(self.n_envs, np.int32)
        check(self.lib.cov_get_n_motion(self.h, ptr(n)))
        return n

    def sync(self):
        check(self.lib.cov_sync(self.h))

    def set_streams(self, n):
        """Launches per step (cov_set_streams): 0 (default) splits the fused greedy steps
        over two HIP streams and launches every other step once; 2 splits every step; 1
        keeps every step on the handle's stream."""
        check(self.lib.cov_set_streams(self.h, int(n)))

    def controller_greedy(self, fetch=True):
        """Greedy expert actions (B,R) int32 and the (B,R) bool mask of robots the
        reference hands to np_random.choice(4); the actions also stay resident for
        step(resident=True). fetch=False leaves both on the device (no sync)."""
        if not fetch:
            check(self.lib.cov_controller_greedy(self.h, None, None, None))
            return None, None
        a = np.empty((self.n_envs, self.n_robots), np.int32)
        rnd = np.empty((self.n_envs, self.n_robots), np.uint8)
        n = ctypes.c_int64()
        check(self.lib.cov_controller_greedy(self.h, ptr(a), ptr(rnd), ctypes.byref(n)))
        return a, rnd.astype(bool)

    def flat_obs(self, f32=False, device_ptr=None):
        """(B, 15*max_nodes + 1) rows in FlattenDictWrapper order (float64 like its
        np.concatenate, or float32). device_ptr: write into that device buffer instead
        (asynchronous on the handle's stream; returns None)."""
        flags = COV_FLAT_F32 if f32 else 0
        if device_ptr is not None:
            check(self.lib.cov_get_flat_obs(self.h, ctypes.c_void_p(int(device_ptr)), flags | COV_OUT_DEVICE))
            return None
        out = np.empty((self.n_envs, 15 * self.max_nodes + 1), np.float32 if f32 else np.float64)
        check(self.lib.cov_get_flat_obs(self.h, ptr(out), flags))
        return out

    def graphs_tuple(self, mask_all=False):
        """unpack_obs (coverage.py:689-741) of the whole batch as host arrays; with
        mask_all every graph drops its padded edges (the reference drops only graph 0's)."""
        flags = COV_MASK_ALL if mask_all else 0
        ne = np.empty(self.n_envs, np.int32)
        tot = ctypes.c_int64()
        check(self.lib.cov_graphs_tuple_sizes(self.h, ptr(ne), ctypes.byref(tot), flags))
        T = int(tot.value)
        o = dict(n_node=np.empty(self.n_envs, np.int32), nodes=np.empty((self.n_envs * self.max_nodes, 3), np.float32),
                 n_edge=np.empty(self.n_envs, np.int32), edges=np.empty((T, 1), np.float32),
                 senders=np.empty(T, np.int32), receivers=np.empty(T, np.int32),
                 globs=np.empty((self.n_envs, 1), np.float32))
        check(self.lib.cov_get_graphs_tuple(self.h, ptr(o["n_node"]), ptr(o["nodes"]), ptr(o["n_edge"]), ptr(o["edges"]),
                                            ptr(o["senders"]), ptr(o["receivers"]), ptr(o["globs"]), flags))
        return o

    def time_matrix(self, env, n_targets):
        """(graph_cost, graph_previous) of one env, each (T,T) int32."""
        c = np.empty((n_targets, n_targets), np.int32)
        p = np.empty((n_targets, n_targets), np.int32)
        check(self.lib.cov_get_time_matrix(self.h, int(env), ptr(c), ptr(p)))
        return c, p


class GraphUtils:
    """Owns one gu_graph context: the radius / k-nearest graph helpers of
    gym_flock/envs/spatial/utils.py (:8-24, :27-39, :60-88) on the device."""

    def __init__(self, device=0):
        self.lib = load()
        h = ctypes.c_void_p()
        check(self.lib.gu_create(device, ctypes.byref(h)))
        self.h = h

    @staticmethod
    def _pos(p):
        p = np.ascontiguousarray(p, dtype=np.float64)
        if p.ndim != 2 or p.shape[1] != 2:
            raise ValueError("positions must be (n, 2), got %s" % (p.shape,))
        return p

    def _edges(self, n):
        E = int(n.value)
        snd = np.empty(E, np.int32)
        rcv = np.empty(E, np.int32)
        r = np.empty(E, np.float64)
        diff = np.empty(2 * E, np.float64)
        check(self.lib.gu_get_edges(self.h, ptr(snd), ptr(rcv), ptr(r), ptr(diff)))
        return snd, rcv, r, diff

    def radius_edges(self, rad, pos1, pos2=None, self_loops=False):
        """(senders, receivers, r, diff) with diff = every dx then every dy."""
        p1 = self._pos(pos1)
        p2 = None if pos2 is None else self._pos(pos2)
        n = ctypes.c_int64()
        check(self.lib.gu_radius_edges(self.h, ptr(p1), len(p1), ptr(p2), 0 if p2 is None else len(p2),
                                       float(rad), int(bool(self_loops)), ctypes.byref(n)))
        return self._edges(n)

    def k_edges(self, k, pos1, pos2=None, self_loops=False, allow_nearest=False):
        p1 = self._pos(pos1)
        p2 = None if pos2 is None else self._pos(pos2)
        n = ctypes.c_int64()
        check(self.lib.gu_k_edges(self.h, int(k), ptr(p1), len(p1), ptr(p2), 0 if p2 is None else len(p2),
                                  int(bool(self_loops)), int(bool(allow_nearest)), ctypes.byref(n)))
        return self._edges(n)

    def nodes_within_radius(self, rad, pos1, pos2):
        p1, p2 = self._pos(pos1), self._pos(pos2)
        valid = np.empty(len(p2), np.uint8)
        check(self.lib.gu_nodes_within_radius(self.h, ptr(p1), len(p1), ptr(p2), len(p2), float(rad), ptr(valid)))
        return valid.astype(bool)

    def close(self):
        if getattr(self, "h", None):
            self.lib.gu_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
