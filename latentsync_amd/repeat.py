"""Integer chunk/frame padding helpers of the window loop -- same semantics as
latentsync/utils/repeat.py:7-258 (used at lipsync_pipeline.py:438-466), pinned
bit-exactly by tests/golden/indices.npz.  Lists of tensors in, lists out; the
audio sample tensor is padded with zeros of its dtype."""
import numpy as np
import torch


def repeat_to_length(array, target_length):
    """repeat.py:7-30 (ceil-div tiling, then truncate)."""
    n = len(array)
    if n >= target_length:
        return array[:target_length]
    k = -(-target_length // n)
    if isinstance(array, torch.Tensor):
        return array.repeat((k, *[1] * (array.dim() - 1)))[:target_length]
    if isinstance(array, np.ndarray):
        return np.tile(array, (k, *[1] * (array.ndim - 1)))[:target_length]
    if isinstance(array, list):
        return (array * k)[:target_length]
    raise TypeError("Unsupported type for repetition")


def truncate_to_length(array, target_length):
    """repeat.py:33-56 (keep the LAST target_length items)."""
    n = len(array)
    if n <= target_length:
        return array
    if isinstance(array, (torch.Tensor, np.ndarray, list)):
        return array[n - target_length:]
    raise TypeError("Unsupported type for truncation")


def _zeros_like_samples(audio, n):
    if isinstance(audio, torch.Tensor):
        return torch.zeros(n, dtype=audio.dtype)
    return np.zeros(n, dtype=np.asarray(audio).dtype)


def _cat(a, b):
    if isinstance(a, torch.Tensor):
        return torch.cat([a, b], 0)
    return np.concatenate([a, b], 0)


def pad_whisper_chunks(chunks, shape, audio, sr, fps=25):
    """repeat.py:81-118: PREPEND zero chunks to a multiple of 16."""
    n = len(chunks)
    k = (16 - n % 16) % 16
    dur = k / fps
    if k > 0:
        chunks = [torch.zeros(shape) for _ in range(k)] + list(chunks)
    pad = int(dur * sr)
    if pad > 0:
        audio = _cat(_zeros_like_samples(audio, pad), audio)
    return chunks, audio, dur, k


def pad_whisper_chunks_end(chunks, shape, audio, sr, fps=25, divisible_by=16):
    """repeat.py:164-209: APPEND zero chunks to a multiple of divisible_by."""
    chunks = list(chunks)
    n = len(chunks)
    k = (divisible_by - n % divisible_by) % divisible_by
    dur = k / fps
    if k > 0:
        chunks = chunks + [torch.zeros(shape) for _ in range(k)]
    audio = audio.clone() if isinstance(audio, torch.Tensor) else np.array(audio, copy=True)
    pad = int(dur * sr)
    if pad > 0:
        audio = _cat(audio, _zeros_like_samples(audio, pad))
    return chunks, audio, dur


def pad_whisper_chunks_to_target(chunks, shape, audio, sr, target_frames, fps=25):
    """repeat.py:211-258: append zero chunks up to target_frames."""
    chunks = list(chunks)
    n = len(chunks)
    if target_frames < n:
        raise ValueError(f"Target frames ({target_frames}) must be greater than or equal to current length ({n})")
    k = target_frames - n
    dur = k / fps
    if k > 0:
        chunks = chunks + [torch.zeros(shape) for _ in range(k)]
    audio = audio.clone() if isinstance(audio, torch.Tensor) else np.array(audio, copy=True)
    pad = int(dur * sr)
    if pad > 0:
        audio = _cat(audio, _zeros_like_samples(audio, pad))
    return chunks, audio, dur
