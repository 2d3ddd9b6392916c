"""configs/unet/*.yaml loading (the reference's UNet constructor schema).

The reference reads its YAML with OmegaConf (scripts/inference.py:110) and passes
``config.model`` as kwargs to ``UNet3DConditionModel`` (unet.py:42-84, 494-496).
OmegaConf is not installed here; PyYAML parses ``norm_eps: 1e-5`` as a *string*
(YAML 1.1), so numeric-looking strings are coerced back to floats exactly as
OmegaConf would ("Config / flags").
"""
import copy
import re

import yaml

_FLOAT_RE = re.compile(r"^[-+]?(\d+\.?\d*|\.\d+)([eE][-+]?\d+)?$")

# LatentSync 1.5 stage-2 UNet topology (configs/unet/stage2.yaml:52-100), used as
# the default model config when no YAML path is given (e.g. on the GPU box,
# where the reference tree does not exist).
STAGE2_MODEL = {
    "act_fn": "silu",
    "add_audio_layer": True,
    "attention_head_dim": 8,
    "block_out_channels": [320, 640, 1280, 1280],
    "center_input_sample": False,
    "cross_attention_dim": 384,
    "down_block_types": ["CrossAttnDownBlock3D", "CrossAttnDownBlock3D", "CrossAttnDownBlock3D", "DownBlock3D"],
    "mid_block_type": "UNetMidBlock3DCrossAttn",
    "up_block_types": ["UpBlock3D", "CrossAttnUpBlock3D", "CrossAttnUpBlock3D", "CrossAttnUpBlock3D"],
    "downsample_padding": 1,
    "flip_sin_to_cos": True,
    "freq_shift": 0,
    "in_channels": 13,
    "layers_per_block": 2,
    "mid_block_scale_factor": 1,
    "norm_eps": 1e-5,
    "norm_num_groups": 32,
    "out_channels": 4,
    "sample_size": 64,
    "resnet_time_scale_shift": "default",
    "use_motion_module": True,
    "motion_module_resolutions": [1, 2, 4, 8],
    "motion_module_mid_block": False,
    "motion_module_decoder_only": False,
    "motion_module_type": "Vanilla",
    "motion_module_kwargs": {
        "num_attention_heads": 8,
        "num_transformer_block": 1,
        "attention_block_types": ["Temporal_Self", "Temporal_Self"],
        "temporal_position_encoding": True,
        "temporal_position_encoding_max_len": 24,
        "temporal_attention_dim_div": 1,
        "zero_initialize": True,
    },
}

# Reduced-width variant used by the parity fixtures.
TINY_MODEL = dict(copy.deepcopy(STAGE2_MODEL), block_out_channels=[32, 64, 64, 64])


def _coerce(v):
    if isinstance(v, str) and _FLOAT_RE.match(v.strip()):
        return float(v)
    if isinstance(v, dict):
        return {k: _coerce(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_coerce(x) for x in v]
    return v


def load_config(path: str) -> dict:
    """Whole YAML file as a dict with OmegaConf-compatible float coercion."""
    with open(path) as f:
        return _coerce(yaml.safe_load(f))


def load_model_config(path: str = None) -> dict:
    """The ``model:`` mapping of a configs/unet/*.yaml file (or STAGE2_MODEL)."""
    if path is None:
        return copy.deepcopy(STAGE2_MODEL)
    cfg = load_config(path)
    return cfg["model"] if "model" in cfg else cfg
