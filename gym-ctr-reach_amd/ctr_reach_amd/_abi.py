"""ctypes binding of libctr_reach_amd.so (the C ABI declared in include/ctr_reach_amd.h).

The library is built in-tree (``python -m ctr_reach_amd.build`` or ``__graft_entry__.build()``)
into ``ctr_reach_amd/lib/``.  There is no CPU fallback: if the shared object is missing or a
call fails, an exception is raised.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CTR_REACH_AMD_LIB") or os.path.join(HERE, "lib", "libctr_reach_amd.so")

CTR_ABI_VERSION = 15
CTR_IPC_HANDLE_BYTES = 64
CTR_GATHER_MAX_RANKS = 16
CTR_MAX_SYSTEMS = 8
CTR_POOL_MAX = 192          # ctr_batch_t.pool_depth limit
CTR_HER_SCAN_TILE = 1024
CTR_INTEGRATOR_RK45_SCIPY = 0
CTR_INTEGRATOR_RK4 = 1
CTR_MODEL_COMPLIANT = 0
CTR_MODEL_RIGID = 1
CTR_STATUS_STEP_UNDERFLOW = 1
CTR_STATUS_SAMPLER_STUCK = 2
CTR_STATUS_NAN = 4
CTR_STATUS_TOO_LONG = 8
CTR_STATUS_POOL_MISS = 16
AUTORESET_OFF = 0        # CTR_AUTORESET_OFF
AUTORESET_SWEEP = 1      # CTR_AUTORESET_SWEEP: pooled resets, misses computed by a sweep launch
AUTORESET_POOLED = 2     # CTR_AUTORESET_POOLED: every reset comes from the pool, no sweep launch
CTR_HER_FUTURE = 0
CTR_HER_FINAL = 1
CTR_HER_EPISODE = 2

_d3 = ctypes.c_double * 3
_P = ctypes.c_void_p


class CtrSystem(ctypes.Structure):
    _fields_ = [("L", _d3), ("Lc", _d3), ("EI", _d3), ("GJ", _d3), ("Ux", _d3), ("Uy", _d3)]


class CtrTubeRaw(ctypes.Structure):
    _fields_ = [("Din", _d3), ("Dout", _d3), ("E", _d3), ("G", _d3)]


class CtrEnvConfig(ctypes.Structure):
    _fields_ = [
        ("n_systems", ctypes.c_int32),
        ("n_substeps", ctypes.c_int32),
        ("max_steps", ctypes.c_int32),
        ("constrain_alpha", ctypes.c_int32),
        ("egocentric", ctypes.c_int32),
        ("resample_joints", ctypes.c_int32),
        ("integrator", ctypes.c_int32),
        ("rk4_steps_per_m", ctypes.c_int32),
        ("model", ctypes.c_int32),
        ("obs_f64", ctypes.c_int32),
        ("tol", ctypes.c_double),
        ("seed", ctypes.c_uint64),
        ("systems", CtrSystem * CTR_MAX_SYSTEMS),
        ("domain_rand", ctypes.c_double),
        ("domain_pad", ctypes.c_double),
        ("raw", CtrTubeRaw * CTR_MAX_SYSTEMS),
    ]


class CtrBatch(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64),
        ("env_base", ctypes.c_int64),
        ("joints", _P),
        ("desired_goal", _P),
        ("achieved_goal", _P),
        ("t", _P),
        ("system", _P),
        ("epoch", _P),
        ("desired_joints", _P),
        ("starting_joints", _P),
        ("starting_position", _P),
        ("work", _P),
        ("work_parity", ctypes.c_int32),
        ("work_pad", ctypes.c_int32),
        ("pool_depth", ctypes.c_int32),
        ("pool_pad", ctypes.c_int32),
        ("pool", _P),             # [P][n] ctr_pool_slot_t, 128 B each (ABI 15)
        ("refill", _P),
        ("refill_cap", ctypes.c_int64),
        ("carry", ctypes.c_void_p),
        ("carry_cap", ctypes.c_int64),
        ("refill_budget", ctypes.c_int32),
        ("refill_lead", ctypes.c_int32),
    ]


class CtrPoolSlot(ctypes.Structure):
    """ctr_pool_slot_t: one precomputed reset, 128 B (ABI 15)."""
    _fields_ = [("dg", ctypes.c_double * 3), ("ag", ctypes.c_double * 3), ("qd", ctypes.c_float * 6),
                ("q0", ctypes.c_float * 6), ("sys", ctypes.c_int32), ("stat", ctypes.c_uint32),
                ("r", ctypes.c_uint32), ("pad", ctypes.c_uint32 * 5)]


# the slot in dwords: [first, last) dword and dtype of every field (the host's strided views)
POOL_SLOT_DWORDS = ctypes.sizeof(CtrPoolSlot) // 4
POOL_SLOT_FIELDS = {
    name: (getattr(CtrPoolSlot, name).offset // 4,
           None if getattr(CtrPoolSlot, name).size == 4 else (getattr(CtrPoolSlot, name).offset +
                                                              getattr(CtrPoolSlot, name).size) // 4,
           kind)
    for name, kind in (("dg", "f64"), ("ag", "f64"), ("qd", "f32"), ("q0", "f32"), ("sys", "i32"), ("stat", "i32"),
                       ("r", "i32"))}
assert POOL_SLOT_DWORDS == 32


class CtrStepOut(ctypes.Structure):
    _fields_ = [
        ("obs", _P),
        ("reward", _P),
        ("done", _P),
        ("success", _P),
        ("error", _P),
        ("terminal_obs", _P),
        ("terminal_achieved", _P),
        ("status", _P),
        ("nfev", _P),
        ("packed", _P),
        ("packed_seq", ctypes.c_uint32),
        ("packed_pad", ctypes.c_uint32),
        ("gather", _P),
        ("gather_prev", _P),
        ("gather_prev_seq", ctypes.c_uint32),
        ("gather_seq", ctypes.c_uint32),
        ("gather_wait_prev", ctypes.c_int32),
        ("gather_pad", ctypes.c_int32),
    ]


class CtrGatherPush(ctypes.Structure):
    _fields_ = [("src", _P), ("n", ctypes.c_int64), ("world", ctypes.c_int32), ("pad", ctypes.c_int32),
                ("dst", _P * CTR_GATHER_MAX_RANKS), ("seqw", _P * CTR_GATHER_MAX_RANKS), ("ticket", _P),
                # fused push flow control (ABI 13; wait_us a wall-clock budget and the poison words: ABI 14)
                ("relw", _P * CTR_GATHER_MAX_RANKS), ("rel", _P), ("wait_seqw", _P), ("err", _P),
                ("depth", ctypes.c_int32), ("wait_us", ctypes.c_uint32),
                ("poisonw", _P * CTR_GATHER_MAX_RANKS), ("poison", _P)]


CTR_GATHER_E_WAIT_TIMEOUT = 1       # a consumer wait gave up
CTR_GATHER_E_OVERWRITTEN = 2        # a sequence word was already past the awaited step
CTR_GATHER_E_RELEASE_TIMEOUT = 4    # a fused push stored into a slot not yet released
CTR_GATHER_E_PREV_TIMEOUT = 8       # the fused consumer wait gave up


class CtrCopy(ctypes.Structure):
    _fields_ = [("dst", _P), ("src", _P), ("bytes", ctypes.c_int64), ("stream", ctypes.c_int32),
                ("pad", ctypes.c_int32)]


class CtrHer(ctypes.Structure):
    _fields_ = [
        ("obs_dim", ctypes.c_int32),
        ("t_max", ctypes.c_int32),
        ("n_sampled_goal", ctypes.c_int32),
        ("strategy", ctypes.c_int32),
        ("n", ctypes.c_int64),
        ("env_base", ctypes.c_int64),
        ("slots", ctypes.c_int32),
        ("pad", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("state", _P),
        ("step", _P),
        ("dg", _P),
        ("tol", _P),
        ("len", _P),
        ("epoch", _P),
        ("cur_t", _P),
        ("cur_epoch", _P),
        ("cdf", _P),
    ]


class CtrHerBatch(ctypes.Structure):
    _fields_ = [("obs", _P), ("action", _P), ("reward", _P), ("next_obs", _P), ("done", _P), ("index", _P)]


EXPORTED = ("ctr_abi_version", "ctr_last_error", "ctr_fk", "ctr_set_action", "ctr_step", "ctr_reset",
            "ctr_pool_refill", "ctr_compute_reward", "ctr_domain_params", "ctr_fk_tables", "ctr_jacobian", "ctr_fk_shape",
            "ctr_her_open", "ctr_her_record", "ctr_her_sample", "ctr_step_her", "ctr_pool_requeue",
            "ctr_ipc_get_handle", "ctr_ipc_open", "ctr_ipc_close", "ctr_seqw_alloc", "ctr_seqw_free", "ctr_copy_list",
            "ctr_gather_wait", "ctr_gather_push", "ctr_gather_publish", "ctr_refill_carry_bytes")

_lib = None


class CtrError(RuntimeError):
    pass


def load(path=None):
    """Load (once) and prototype the shared library.  Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or LIB_PATH
    if not os.path.exists(path):
        raise CtrError("libctr_reach_amd.so not built (%s); run __graft_entry__.build()" % path)
    L = ctypes.CDLL(path)
    i64, i32 = ctypes.c_int64, ctypes.c_int32
    L.ctr_abi_version.restype = ctypes.c_int
    L.ctr_last_error.restype = ctypes.c_char_p
    L.ctr_fk.argtypes = [_P, _P, i64, ctypes.POINTER(CtrEnvConfig), _P, _P, _P, _P]
    L.ctr_set_action.argtypes = [ctypes.POINTER(CtrEnvConfig), _P, _P, _P, i64, _P]
    L.ctr_step.argtypes = [ctypes.POINTER(CtrEnvConfig), ctypes.POINTER(CtrBatch), _P,
                           ctypes.POINTER(CtrStepOut), i32, _P]
    L.ctr_reset.argtypes = [ctypes.POINTER(CtrEnvConfig), ctypes.POINTER(CtrBatch), _P, _P, _P, _P, _P, _P]
    L.ctr_pool_refill.argtypes = [ctypes.POINTER(CtrEnvConfig), ctypes.POINTER(CtrBatch), _P]
    L.ctr_pool_requeue.argtypes = [ctypes.POINTER(CtrEnvConfig), ctypes.POINTER(CtrBatch), _P]
    L.ctr_compute_reward.argtypes = [_P, _P, i64, ctypes.c_double, _P, _P]
    L.ctr_domain_params.argtypes = [ctypes.POINTER(CtrEnvConfig), ctypes.POINTER(CtrBatch), _P, _P, _P]
    L.ctr_fk_tables.argtypes = [_P, _P, i64, ctypes.POINTER(CtrEnvConfig), _P, _P, _P, _P]
    L.ctr_fk_shape.argtypes = [_P, _P, _P, i64, ctypes.POINTER(CtrEnvConfig), i32, _P, _P, _P, _P, _P, _P]
    L.ctr_jacobian.argtypes = [_P, _P, i64, ctypes.POINTER(CtrEnvConfig), ctypes.c_double, _P, _P, _P, _P]
    L.ctr_her_open.argtypes = [ctypes.POINTER(CtrHer), ctypes.POINTER(CtrBatch), _P, _P, _P]
    L.ctr_her_record.argtypes = [ctypes.POINTER(CtrHer), ctypes.POINTER(CtrBatch), _P, ctypes.POINTER(CtrStepOut),
                                 ctypes.c_double, _P]
    L.ctr_her_sample.argtypes = [ctypes.POINTER(CtrHer), i64, ctypes.c_uint64, ctypes.c_uint64,
                                 ctypes.POINTER(CtrHerBatch), _P]
    L.ctr_step_her.argtypes = [ctypes.POINTER(CtrEnvConfig), ctypes.POINTER(CtrBatch), _P,
                               ctypes.POINTER(CtrStepOut), i32, ctypes.POINTER(CtrHer), _P]
    try:           # ABI 11 (an allowed older A/B build lacks them)
        L.ctr_ipc_get_handle.argtypes = [_P, _P]
        L.ctr_ipc_open.argtypes = [_P, ctypes.POINTER(_P)]
        L.ctr_ipc_close.argtypes = [_P]
        L.ctr_seqw_alloc.argtypes = [i64, ctypes.POINTER(_P)]
        L.ctr_seqw_free.argtypes = [_P]
        L.ctr_copy_list.argtypes = [ctypes.POINTER(CtrCopy), i32, ctypes.POINTER(_P), i32, _P, ctypes.POINTER(_P)]
        L.ctr_gather_wait.argtypes = [_P, i32, ctypes.c_uint32, ctypes.c_uint32, _P, _P]
        L.ctr_gather_push.argtypes = [ctypes.POINTER(CtrGatherPush), ctypes.c_uint32, i32, _P]
        L.ctr_gather_publish.argtypes = [_P, ctypes.c_uint32, _P]
    except AttributeError:
        if L.ctr_abi_version() == CTR_ABI_VERSION:
            raise
    for fn in EXPORTED[2:]:
        if hasattr(L, fn):
            getattr(L, fn).restype = ctypes.c_int
    if hasattr(L, "ctr_refill_carry_bytes"):       # ABI 12
        L.ctr_refill_carry_bytes.argtypes = [i64]
        L.ctr_refill_carry_bytes.restype = i64
    # A/B timing of an older build (tools/experiments/build_rev.sh) may name its ABI version in
    # CTR_REACH_AMD_ALLOW_ABI; only entry points both versions share may then be called
    allowed = {CTR_ABI_VERSION, int(os.environ.get("CTR_REACH_AMD_ALLOW_ABI", CTR_ABI_VERSION))}
    if L.ctr_abi_version() not in allowed:
        raise CtrError("ABI version mismatch: library %d, binding %d" % (L.ctr_abi_version(), CTR_ABI_VERSION))
    _lib = L
    return L


def check(rc, what):
    if rc != 0:
        msg = _lib.ctr_last_error().decode() if _lib is not None else ""
        raise CtrError("%s failed (rc=%d): %s" % (what, rc, msg))


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None, device_index=None):
    """hipStream_t of `stream`, or of the current stream of `device_index` (default: the current
    device).  The current-stream path reads the raw handle directly (torch.cuda.current_stream()
    builds a Stream object, ~3 us a call, a fifth of a small batch's step)."""
    import torch
    if stream is not None:
        return ctypes.c_void_p(stream.cuda_stream)
    if device_index is None:
        device_index = torch.cuda.current_device()
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(device_index))
