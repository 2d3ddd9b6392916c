"""ctypes binding of libls_hip.so (include/ls_hip.h).

This is the only door from the host package to the kernels.  There is no
fallback: if the library is missing or was built for another ABI, importing
the product path raises immediately (loud failure is part of the parity
contract -- a silent CPU/eager fallback would void every GPU parity claim).
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LS_HIP_LIB", os.path.join(HERE, "libls_hip.so"))
ABI_VERSION = 13



def ab_switch(name: str, default: str) -> str:
    """An A/B switch of the host dispatch, read from the environment ONLY in diagnostics
    mode (LS_DIAG_BUILD=1, the same flag that builds the library's A/B kernels): the
    default product path does not depend on the environment."""
    if os.environ.get("LS_DIAG_BUILD", "") in ("", "0"):
        return default
    return os.environ.get(name, default)


c_u16p = C.c_void_p
c_vp = C.c_void_p


class ConvDesc(C.Structure):
    _fields_ = [
        ("x1", c_vp), ("x2", c_vp),
        ("C1", C.c_int32), ("C2", C.c_int32),
        ("ld1", C.c_int32), ("ld2", C.c_int32),
        ("n_img", C.c_int32), ("H", C.c_int32), ("W", C.c_int32),
        ("Ho", C.c_int32), ("Wo", C.c_int32),
        ("ksize", C.c_int32), ("stride", C.c_int32), ("pad", C.c_int32), ("upsample", C.c_int32),
        ("aff_scale", c_vp), ("aff_shift", c_vp), ("imgs_per_sample", C.c_int32), ("silu_in", C.c_int32),
        ("w", c_vp), ("K", C.c_int32), ("N", C.c_int32),
        ("bias", c_vp),
        ("rowvec", c_vp), ("rows_per_vec", C.c_int32), ("rowvec_ld", C.c_int32),
        ("res", c_vp), ("ldr", C.c_int32), ("out_scale", C.c_float),
        ("act", C.c_int32),
        ("y", c_vp), ("ldy", C.c_int32), ("y_f32", C.c_int32),
        ("split_k", C.c_int32),
        ("workspace", c_vp), ("workspace_bytes", C.c_size_t),
        ("ln_rowstats", c_vp), ("ln_colsum", c_vp), ("rowvec_mod", C.c_int32),
        ("row_stats_out", c_vp), ("row_stats_eps", C.c_float),
        ("gn_colsum_out", c_vp),
    ]


class AttnDesc(C.Structure):
    _fields_ = [("q", c_vp), ("k", c_vp), ("v", c_vp), ("o", c_vp)] + [
        (f"{t}_{s}", C.c_int64) for t in "qkvo" for s in ("sb1", "sb2", "si", "sh")
    ] + [
        ("batch", C.c_int32), ("z2", C.c_int32), ("heads", C.c_int32), ("nq", C.c_int32),
        ("nk", C.c_int32), ("head_dim", C.c_int32), ("scale", C.c_float),
    ]


class TAttnDesc(C.Structure):
    _fields_ = [("x", c_vp), ("ldx", C.c_int32), ("gamma", c_vp), ("bpe", c_vp), ("w", c_vp), ("o", c_vp),
                ("ldo", C.c_int32), ("C", C.c_int32), ("heads", C.c_int32), ("n_samples", C.c_int32),
                ("F", C.c_int32), ("S", C.c_int32), ("eps", C.c_float)]


class FFDesc(C.Structure):
    _fields_ = [("x", c_vp), ("ln_rowstats", c_vp), ("w1", c_vp), ("b1", c_vp), ("w2", c_vp), ("b2", c_vp),
                ("y", c_vp), ("M", C.c_int64), ("ldx", C.c_int32), ("ldy", C.c_int32), ("C", C.c_int32),
                ("inner", C.c_int32)]


class FFChainDesc(C.Structure):
    _fields_ = [("o", c_vp), ("wo", c_vp), ("bo", c_vp), ("h1", c_vp), ("w1", c_vp), ("b1", c_vp), ("w2", c_vp),
                ("b2", c_vp), ("wp", c_vp), ("bp", c_vp), ("xb", c_vp), ("z", c_vp), ("cs_out", c_vp),
                ("M", C.c_int64), ("ldo", C.c_int32), ("ldh", C.c_int32), ("ldxb", C.c_int32), ("ldz", C.c_int32),
                ("C", C.c_int32), ("inner", C.c_int32), ("eps", C.c_float)]


class XAttnDesc(C.Structure):
    _fields_ = [("x", c_vp), ("ln_rowstats", c_vp), ("wq", c_vp), ("bq", c_vp), ("kv", c_vp), ("wo", c_vp),
                ("bo", c_vp), ("y", c_vp), ("stats_out", c_vp), ("M", C.c_int64), ("ldx", C.c_int32),
                ("ldy", C.c_int32), ("ldkv", C.c_int32), ("C", C.c_int32), ("heads", C.c_int32), ("L", C.c_int32),
                ("hw", C.c_int32), ("eps", C.c_float)]


_SIGS = {
    "ls_abi_version": (C.c_int, []),
    "ls_last_error": (C.c_char_p, []),
    "ls_conv2d": (C.c_int, [C.POINTER(ConvDesc), c_vp]),
    "ls_conv_workspace_bytes": (C.c_size_t, [C.POINTER(ConvDesc)]),
    "ls_conv_path": (C.c_int, [C.POINTER(ConvDesc)]),
    "ls_groupnorm": (C.c_int, [c_vp, c_vp, C.c_int32, C.c_int32, C.c_int32, C.c_int64, C.c_int32, C.c_float,
                               c_vp, c_vp, c_vp, c_vp, c_vp, C.c_size_t, c_vp]),
    "ls_groupnorm_workspace_bytes": (C.c_size_t, [C.c_int32, C.c_int32]),
    "ls_groupnorm_colsum": (C.c_int, [c_vp, c_vp, C.c_int32, C.c_int32, C.c_int32, C.c_int64, C.c_int32, C.c_float,
                                      c_vp, c_vp, c_vp, c_vp, c_vp]),
    "ls_gn_colsum": (C.c_int, [c_vp, C.c_int64, C.c_int64, C.c_int32, c_vp, c_vp]),
    "ls_groupnorm_apply": (C.c_int, [c_vp, c_vp, C.c_int32, C.c_int32, C.c_int64, C.c_int64, c_vp, c_vp, C.c_int32,
                                     c_vp, c_vp]),
    "ls_layernorm": (C.c_int, [c_vp, C.c_int64, C.c_int64, C.c_int32, C.c_float, c_vp, c_vp, c_vp, C.c_int32, C.c_int32,
                               c_vp, c_vp]),
    "ls_row_stats": (C.c_int, [c_vp, C.c_int64, C.c_int64, C.c_int32, C.c_float, c_vp, c_vp]),
    "ls_attention": (C.c_int, [C.POINTER(AttnDesc), c_vp]),
    "ls_attention_fp8_workspace_bytes": (C.c_size_t, [C.POINTER(AttnDesc)]),
    "ls_attention_fp8": (C.c_int, [C.POINTER(AttnDesc), c_vp, C.c_size_t, c_vp]),
    "ls_temporal_attention": (C.c_int, [C.POINTER(TAttnDesc), c_vp]),
    "ls_feedforward": (C.c_int, [C.POINTER(FFDesc), c_vp]),
    "ls_cross_attention_block": (C.c_int, [C.POINTER(XAttnDesc), c_vp]),
    "ls_ff_chain": (C.c_int, [C.POINTER(FFChainDesc), c_vp]),
    "ls_small_linear": (C.c_int, [c_vp, C.c_int32, C.c_int32, c_vp, c_vp, C.c_int32, C.c_int32, c_vp, c_vp]),
    "ls_timestep_embed": (C.c_int, [c_vp, c_vp, C.c_int32, C.c_int32, C.c_int32, C.c_float, c_vp, c_vp]),
    "ls_timestep_embed_f32": (C.c_int, [c_vp, C.c_int32, C.c_int32, C.c_int32, C.c_float, c_vp, c_vp]),
    "ls_ddim_cfg_step": (C.c_int, [c_vp, C.c_int32, C.c_int32, C.c_int64, C.c_float, c_vp, c_vp, c_vp, c_vp,
                                   C.c_int32, c_vp]),
    "ls_prep_pixels": (C.c_int, [c_vp, C.c_int32, C.c_int32, c_vp, c_vp, c_vp, C.c_int32, c_vp]),
    "ls_vae_sample": (C.c_int, [c_vp, C.c_int32, c_vp, C.c_int64, C.c_float, C.c_float, c_vp, C.c_int32,
                                C.c_int32, c_vp]),
    "ls_pack_unet_input": (C.c_int, [c_vp, c_vp, c_vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, c_vp,
                                     C.c_int32, c_vp]),
    "ls_scale_latents": (C.c_int, [c_vp, C.c_int64, C.c_float, C.c_float, c_vp, C.c_int32, c_vp]),
    "ls_paste_back": (C.c_int, [c_vp, C.c_int32, c_vp, C.c_int32, c_vp, C.c_int32, C.c_int32, c_vp, c_vp, c_vp]),
    "ls_set_tuning": (C.c_int, [C.c_int32, C.c_int32]),
    "ls_gemm_occupancy": (C.c_int, [C.c_int32]),
    "ls_log_mel_workspace_bytes": (C.c_size_t, [C.c_int64, C.c_int32]),
    "ls_log_mel": (C.c_int, [c_vp, C.c_int64, c_vp, C.c_int32, C.c_int64, c_vp, c_vp, C.c_size_t, c_vp]),
    "ls_audio_chunks": (C.c_int, [c_vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_double,
                                  C.c_int32, C.c_int32, c_vp, C.c_int32, c_vp]),
    "ls_face_resize_u8": (C.c_int, [c_vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, c_vp, c_vp]),
    "ls_restore_tables_bytes": (C.c_size_t, [C.c_int32]),
    "ls_restore_init_tables": (C.c_int, [c_vp, C.c_int32, c_vp]),
    "ls_restore_workspace_bytes": (C.c_size_t, [C.c_int32, C.c_int32, C.c_int32]),
    "ls_restore_frames": (C.c_int, [c_vp, C.c_int32, C.c_int32, C.c_int32, c_vp, C.c_int32, C.c_int32, c_vp, c_vp,
                                    C.c_int32, C.c_int32, C.c_int32, c_vp, c_vp, C.c_size_t, c_vp]),
    "ls_resize_lanczos4_workspace_bytes": (C.c_size_t, [C.c_int32, C.c_int32]),
    "ls_resize_lanczos4_u8": (C.c_int, [c_vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, c_vp, C.c_int32, C.c_int32,
                                        c_vp, C.c_size_t, c_vp]),
    "ls_align_warp_u8": (C.c_int, [c_vp, C.c_int32, C.c_int32, C.c_int32, c_vp, C.c_int32, C.c_int32, C.c_int32,
                                   c_vp, c_vp, c_vp]),
    "ls_add_rows": (C.c_int, [c_vp, C.c_int64, C.c_int32, C.c_int32, c_vp, C.c_int32, c_vp, C.c_int32, c_vp]),
}

EXPORTED = tuple(_SIGS)

_lib = None


def load(path: str = None):
    """Load (once) and type the library.  Raises if it is missing or stale."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("LS_HIP_LIB") or LIB_PATH  # LS_HIP_LIB: A/B builds in tools
    # torch first: its wheel bundles a HIP runtime with the same soname
    # (libamdhip64.so.7) as /opt/rocm's.  Loaded in this order the library binds to
    # torch's runtime, so torch's streams and allocations are valid for the kernels;
    # loaded first, it would pull in the second runtime and launches fail with
    # "no ROCm-capable device is detected" (gpurun_out/r01f_smoke.log).
    import torch  # noqa: F401
    if not os.path.exists(path):
        raise RuntimeError(f"libls_hip.so not found at {path}: run `python -m latentsync_amd.build` "
                           "(the HIP library is required; there is no fallback path)")
    lib = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.ls_abi_version() != ABI_VERSION:
        raise RuntimeError(f"libls_hip.so ABI {lib.ls_abi_version()} != {ABI_VERSION}; rebuild it")
    # diagnostics A/B runs: LS_TUNE="key=value,..." applied through ls_set_tuning
    for kv in filter(None, ab_switch("LS_TUNE", "").split(",")):
        k, v = (int(t) for t in kv.split("="))
        if lib.ls_set_tuning(k, v) != 0:
            raise RuntimeError(f"LS_TUNE {kv}: {lib.ls_last_error().decode()}")
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = _lib.ls_last_error().decode() if _lib is not None else ""
        raise RuntimeError(f"{what} failed (status {rc}): {msg}")
