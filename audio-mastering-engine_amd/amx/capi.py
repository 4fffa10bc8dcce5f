"""ctypes binding of libamx.so (include/amx.h).

The product's only compute path: every per-sample stage runs in the HIP kernels
behind this ABI.  If the library is missing this module raises -- there is no
CPU fallback.
"""
import ctypes
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libamx.so")

c_double_p = ctypes.POINTER(ctypes.c_double)
c_float_p = ctypes.POINTER(ctypes.c_float)

AMX_OK, AMX_EINVAL, AMX_EHIP, AMX_ENOMEM, AMX_ERANGE = 0, -1, -2, -3, -4
ABI_VERSION = 4
CTL_FAST = 1
MODES = ("off", "skip", "linear", "dynamic")
STATS = 16
UP_EDGE = 80      # frames of a neighbour rank the 192 kHz resampler window reaches (amx_internal.hpp)
STAGES = ("front1", "scan_eq", "front2", "scan_xo", "xover", "rms", "env", "fix", "apply")


class AmxError(RuntimeError):
    pass


class ChainDesc(ctypes.Structure):
    _fields_ = [
        ("sample_rate", ctypes.c_int32), ("channels_in", ctypes.c_int32),
        ("input_s16", ctypes.c_int32), ("measure_only", ctypes.c_int32),
        ("analog_on", ctypes.c_int32), ("analog_drive", ctypes.c_float),
        ("tanh_lut", c_float_p),
        ("analog_lo_ba", ctypes.c_double * 6), ("analog_lo_gain", ctypes.c_double),
        ("analog_hi_ba", ctypes.c_double * 6), ("analog_hi_gain", ctypes.c_double),
        ("eq_kind", ctypes.c_int32 * 4), ("eq_gain_db", ctypes.c_double * 4),
        ("eq_gain", ctypes.c_double * 4), ("eq_coef", (ctypes.c_double * 24) * 4),
        ("width_on", ctypes.c_int32), ("width", ctypes.c_float),
        ("multiband_on", ctypes.c_int32),
        ("xover_lo_sos", ctypes.c_double * 12), ("xover_hi_sos", ctypes.c_double * 12),
        ("comp_threshold_db", ctypes.c_double * 3), ("comp_ratio", ctypes.c_double * 3),
        ("comp_m_table", c_double_p * 3),
        ("env_warm_frames", ctypes.c_int32), ("env_rounds", ctypes.c_int32),
        ("stream_chain", ctypes.c_int32), ("pad_sc_", ctypes.c_int32), ("eq_in_lut", c_float_p),
    ]


class Chunk(ctypes.Structure):
    _fields_ = [("track", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("in_offset", ctypes.c_int64), ("frames", ctypes.c_int64)]


class FinalDesc(ctypes.Structure):
    _fields_ = [("limit", ctypes.c_double), ("attack_ms", ctypes.c_double),
                ("release_ms", ctypes.c_double), ("level_in", ctypes.c_double),
                ("level_out", ctypes.c_double), ("auto_level", ctypes.c_int32),
                ("from_rest", ctypes.c_int32)]


class DecideDesc(ctypes.Structure):
    _fields_ = [("lufs_on", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("target_i", ctypes.c_double), ("target_tp", ctypes.c_double),
                ("target_lra", ctypes.c_double)]


class PlanInfo(ctypes.Structure):
    _fields_ = [("workspace_bytes", ctypes.c_int64), ("out_frames", ctypes.c_int64),
                ("n_tracks", ctypes.c_int32), ("n_chunks", ctypes.c_int32),
                ("n_segments", ctypes.c_int64), ("seg_frames", ctypes.c_int32),
                ("scan_levels_eq", ctypes.c_int32), ("scan_levels_xover", ctypes.c_int32),
                ("scan_levels_kw", ctypes.c_int32), ("eq_dim", ctypes.c_int32),
                ("hop_frames", ctypes.c_int32), ("meas_rate", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("max_hops", ctypes.c_int64)]


class LoudnormDesc(ctypes.Structure):
    _fields_ = [(k, ctypes.c_double) for k in ("target_i", "target_lra", "target_tp", "measured_i",
                                                 "measured_lra", "measured_tp", "measured_thresh", "offset")] + \
        [("reuse_stream", ctypes.c_int32)]


class LnShard(ctypes.Structure):
    _fields_ = [("part", ctypes.c_int32), ("kb", ctypes.c_int32), ("ke", ctypes.c_int32), ("windowed", ctypes.c_int32),
                ("u_lo", ctypes.c_int64), ("u_hi", ctypes.c_int64), ("d_rec_in", ctypes.c_void_p),
                ("d_rec_out", ctypes.c_void_p)]


class FlacInfo(ctypes.Structure):
    _fields_ = [("sample_rate", ctypes.c_int32), ("channels", ctypes.c_int32),
                ("bits_per_sample", ctypes.c_int32), ("max_block", ctypes.c_int32),
                ("total_frames", ctypes.c_int64)]


class TrackSpan(ctypes.Structure):
    _fields_ = [("out_offset", ctypes.c_int64), ("out_frames", ctypes.c_int64),
                ("track_frame0", ctypes.c_int64), ("track_frames_total", ctypes.c_int64)]


# every symbol include/amx.h declares (checked by the CPU test suite)
EXPORTS = ("amx_abi_version", "amx_last_error", "amx_build_id", "amx_plan_create", "amx_plan_free",
           "amx_plan_get_info", "amx_plan_track_span", "amx_run_chunks", "amx_run_stage",
           "amx_loudness_pass1", "amx_loudness_pass1_part",
           "amx_kw_propagate", "amx_loudness_pass2", "amx_loudness_histograms",
           "amx_limiter_geometry", "amx_limiter_prepare", "amx_loudness_decide", "amx_kw_carry_setup", "amx_kw_carry", "amx_kw_carry_rows", "amx_plan_set_publish",
           "amx_finalize", "amx_env_counters", "amx_pcm_to_s16", "amx_loudnorm_192k_size",
           "amx_loudnorm_192k", "amx_loudnorm_192k_ex", "amx_flac_info", "amx_flac_decode",
           "amx_plan_set_gate", "amx_loudnorm_192k_shard", "amx_loudnorm_192k_segments",
           "amx_loudnorm_192k_shard_window", "amx_publish_ctl", "amx_plan_set_limiter_trace",
           "amx_mc_plan_create", "amx_mc_plan_free", "amx_mc_plan_get_info", "amx_mc_run_chunks",
           "amx_mc_split_pairs", "amx_mc_loudness_combine", "amx_mc_peak_pick", "amx_mc_limiter_out")
PCM_FORMATS = {"u8": 0, "s16": 1, "s24": 2, "s32": 3, "f32": 4, "f64": 5,
               "s8": 6, "s16be": 7, "s24be": 8, "s32be": 9, "f32be": 10, "f64be": 11}

_lib = None


def load(path=None):
    """Load libamx.so (built in-tree by __graft_entry__.build()); raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or os.environ.get("AMX_LIB") or LIB_PATH     # AMX_LIB: a variant build (experiments)
    if not os.path.exists(p):
        raise AmxError("libamx.so not found at %s -- build it with "
                       "`python -c 'import __graft_entry__ as g; g.build()'`" % p)
    L = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
    vp = ctypes.c_void_p
    L.amx_abi_version.restype = ctypes.c_int
    L.amx_last_error.restype = ctypes.c_char_p
    L.amx_plan_create.argtypes = [ctypes.POINTER(ChainDesc), ctypes.POINTER(Chunk), ctypes.c_int32,
                                  ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                  ctypes.c_int32, ctypes.POINTER(vp)]
    L.amx_plan_free.argtypes = [vp]
    L.amx_plan_free.restype = None
    L.amx_plan_get_info.argtypes = [vp, ctypes.POINTER(PlanInfo)]
    L.amx_plan_track_span.argtypes = [vp, ctypes.c_int32, ctypes.POINTER(TrackSpan)]
    L.amx_run_chunks.argtypes = [vp, vp, vp, vp, vp]
    L.amx_run_stage.argtypes = [vp, ctypes.c_int32, vp, vp, vp, vp]
    L.amx_loudness_pass1.argtypes = [vp, vp, vp, vp, vp, vp, vp]
    L.amx_loudness_pass1_part.argtypes = [vp, ctypes.c_int32, vp, vp, vp, vp, vp, vp]
    L.amx_pcm_to_s16.argtypes = [vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, vp, vp]
    L.amx_env_counters.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]
    L.amx_plan_set_gate.argtypes = [vp, vp]
    L.amx_plan_set_limiter_trace.argtypes = [vp, vp]
    L.amx_mc_plan_create.argtypes = [ctypes.POINTER(ChainDesc), ctypes.POINTER(Chunk), ctypes.c_int32,
                                     ctypes.c_int32, ctypes.POINTER(vp)]
    L.amx_mc_plan_free.argtypes = [vp]
    L.amx_mc_plan_free.restype = None
    L.amx_mc_plan_get_info.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    L.amx_mc_run_chunks.argtypes = [vp, vp, vp, vp, vp]
    L.amx_mc_split_pairs.argtypes = [vp, ctypes.c_int64, ctypes.c_int32, vp, vp]
    L.amx_mc_loudness_combine.argtypes = [vp, ctypes.c_int64, vp, ctypes.c_int32, vp, vp, vp]
    L.amx_mc_peak_pick.argtypes = [vp, ctypes.c_int64, ctypes.c_int32, vp, vp, vp]
    L.amx_mc_limiter_out.argtypes = [vp, ctypes.POINTER(FinalDesc), vp, ctypes.c_int32, vp, vp, vp, vp, vp]
    L.amx_kw_propagate.argtypes = [vp, ctypes.c_int64, c_double_p, c_double_p]
    L.amx_loudness_pass2.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int64, vp, vp]
    L.amx_loudness_histograms.argtypes = [vp, vp, ctypes.c_int64, vp, vp, vp, vp]
    L.amx_limiter_geometry.argtypes = [vp, ctypes.POINTER(FinalDesc), ctypes.POINTER(ctypes.c_int32),
                                       ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)]
    L.amx_limiter_prepare.argtypes = [vp, ctypes.POINTER(FinalDesc), ctypes.c_int32, ctypes.c_int32]
    L.amx_loudness_decide.argtypes = [vp, ctypes.POINTER(DecideDesc), ctypes.POINTER(FinalDesc),
                                      vp, vp, vp, vp, vp, vp, vp]
    L.amx_kw_carry_setup.argtypes = [vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]
    L.amx_kw_carry.argtypes = [vp, vp, vp, vp]
    L.amx_kw_carry_rows.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp]
    L.amx_plan_set_publish.argtypes = [vp, vp]
    L.amx_finalize.argtypes = [vp, ctypes.POINTER(FinalDesc), vp, vp, vp, ctypes.c_int32, vp, vp,
                               vp, vp, vp]
    L.amx_loudnorm_192k_size.argtypes = [vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64),
                                         ctypes.POINTER(ctypes.c_int64)]
    L.amx_loudnorm_192k.argtypes = [vp, ctypes.c_int32, ctypes.POINTER(LoudnormDesc), vp, vp,
                                    ctypes.c_int64, vp, vp, vp, vp, vp]
    L.amx_loudnorm_192k_ex.argtypes = [vp, ctypes.c_int32, ctypes.POINTER(LoudnormDesc), vp, vp, vp, vp, vp,
                                       ctypes.c_int64, vp, vp, vp, vp, vp]
    L.amx_loudnorm_192k_shard.argtypes = [vp, ctypes.c_int32, ctypes.POINTER(LoudnormDesc), vp, vp,
                                          ctypes.POINTER(LnShard), vp, vp, ctypes.c_int64, vp, vp, vp, vp, vp]
    L.amx_publish_ctl.argtypes = [vp, vp, ctypes.c_int32, vp]
    L.amx_loudnorm_192k_shard_window.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                 ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    L.amx_loudnorm_192k_segments.argtypes = [vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), ctypes.c_int32,
                                             ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                             ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)]
    L.amx_flac_info.argtypes = [vp, ctypes.c_int64, ctypes.POINTER(FlacInfo)]
    L.amx_flac_decode.argtypes = [vp, ctypes.c_int64, vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                  ctypes.c_int32, vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    if L.amx_abi_version() != ABI_VERSION:
        raise AmxError("libamx ABI version mismatch")
    L.amx_build_id.restype = ctypes.c_char_p
    stamp = L.amx_build_id().decode()
    if p == LIB_PATH:
        # provenance: the in-tree library must be compiled from the sources of this tree
        from . import build
        want = build.source_hash()
        if stamp != want:
            raise AmxError("libamx.so at %s was built from sources %s, this tree's are %s: "
                           "rebuild it (amx.build.build())" % (p, stamp[:16], want[:16]))
    _lib = L
    return L


def build_id():
    """the source hash stamped into the loaded library (amx_build_id)"""
    return load().amx_build_id().decode()


def check(rc, what):
    if rc != AMX_OK:
        msg = load().amx_last_error()
        raise AmxError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))


def ptr(t):
    """Device pointer of a torch tensor (or None)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def ptr_stream(stream=None):
    """hipStream_t of a torch stream (default: the current one) for the C ABI."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class Plan:
    """Owns an amx_plan*; see include/amx.h for the call contract."""

    def __init__(self, desc, chunks, track_frame0=None, track_total=None, seg_frames=128):
        L = load()
        arr = (Chunk * max(1, len(chunks)))()
        for i, (t, off, n) in enumerate(chunks):
            arr[i].track, arr[i].in_offset, arr[i].frames = int(t), int(off), int(n)
        nt = (max(c[0] for c in chunks) + 1) if chunks else 0
        f0 = (ctypes.c_int64 * max(1, nt))(*(track_frame0 or [0] * nt)) if track_frame0 else None
        tt = (ctypes.c_int64 * max(1, nt))(*track_total) if track_total else None
        h = ctypes.c_void_p()
        self._desc = desc  # keep tables referenced by pointer alive
        check(L.amx_plan_create(ctypes.byref(desc), arr, len(chunks), f0, tt, int(seg_frames),
                                ctypes.byref(h)), "amx_plan_create")
        self.h = h
        info = PlanInfo()
        check(L.amx_plan_get_info(h, ctypes.byref(info)), "amx_plan_get_info")
        self.info = info

    def span(self, track):
        s = TrackSpan()
        check(load().amx_plan_track_span(self.h, int(track), ctypes.byref(s)), "amx_plan_track_span")
        return s

    def kw_propagate(self, frames, state8):
        import numpy as np
        a = np.ascontiguousarray(state8, np.float64).reshape(8)
        out = np.zeros(8, np.float64)
        check(load().amx_kw_propagate(self.h, int(frames), a.ctypes.data_as(c_double_p),
                                      out.ctypes.data_as(c_double_p)), "amx_kw_propagate")
        return out

    def kw_carry_setup(self, frames_after):
        n = len(frames_after)
        arr = (ctypes.c_int64 * max(1, n))(*[int(f) for f in frames_after])
        check(load().amx_kw_carry_setup(self.h, n, arr), "amx_kw_carry_setup")

    def set_publish(self, host):
        """amx_plan_set_publish: a pinned host int32 tensor k_decide also stores the
        decision words into (None: stop)"""
        check(load().amx_plan_set_publish(self.h, ctypes.c_void_p(host.data_ptr()) if host is not None else None),
              "amx_plan_set_publish")

    def set_gate(self, d_word):
        """amx_plan_set_gate: a device int32 tensor (its first word), or None"""
        check(load().amx_plan_set_gate(self.h, ptr(d_word) if d_word is not None else None), "amx_plan_set_gate")

    def limiter_geometry(self, fd):
        bs, halo, sd = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        check(load().amx_limiter_geometry(self.h, ctypes.byref(fd), ctypes.byref(bs),
                                          ctypes.byref(halo), ctypes.byref(sd)),
              "amx_limiter_geometry")
        return bs.value, halo.value, sd.value

    def limiter_prepare(self, fd, seg_frames=0, warm_frames=-1):
        """General-path limiter segments (<= 0: the library default, 16384 frames) and
        their warm-up (< 0: the library default, 3 releases + the ring)."""
        check(load().amx_limiter_prepare(self.h, ctypes.byref(fd), int(seg_frames), int(warm_frames)),
              "amx_limiter_prepare")

    def close(self):
        if getattr(self, "h", None):
            load().amx_plan_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class McPlan:
    """Owns an amx_mc_plan* (a file with 3..8 channels; include/amx.h)."""

    def __init__(self, desc, chunks, seg_frames=128):
        L = load()
        arr = (Chunk * max(1, len(chunks)))()
        for i, (t, off, n) in enumerate(chunks):
            arr[i].track, arr[i].in_offset, arr[i].frames = int(t), int(off), int(n)
        h = ctypes.c_void_p()
        self._desc = desc
        check(L.amx_mc_plan_create(ctypes.byref(desc), arr, len(chunks), int(seg_frames), ctypes.byref(h)),
              "amx_mc_plan_create")
        self.h = h
        ws, nout = ctypes.c_int64(), ctypes.c_int64()
        check(L.amx_mc_plan_get_info(h, ctypes.byref(ws), ctypes.byref(nout)), "amx_mc_plan_get_info")
        self.workspace_bytes, self.out_frames = ws.value, nout.value

    def close(self):
        if getattr(self, "h", None):
            load().amx_mc_plan_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
