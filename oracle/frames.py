"""Synthetic frame hash restated in numpy (TEST INFRASTRUCTURE ONLY).

Frame (scene, state) is ``frame_bytes / 4`` little-endian uint32 words,
word w = hash(scene, state, w) (DESIGN.md "Synthetic scenes").
"""
import numpy as np


def frame_hash(scene, state, w):
    scene = np.uint32(scene)
    state = np.asarray(state, dtype=np.uint32)
    w = np.asarray(w, dtype=np.uint32)
    with np.errstate(over="ignore"):
        x = (w * np.uint32(0x9E3779B1)) ^ (state * np.uint32(0x85EBCA77)) ^ (scene * np.uint32(0xC2B2AE3D)) ^ np.uint32(0x27D4EB2F)
        x ^= x >> np.uint32(16)
        x *= np.uint32(0x7FEB352D)
        x ^= x >> np.uint32(15)
        x *= np.uint32(0x846CA68B)
        x ^= x >> np.uint32(16)
    return x


def synth_frames(scene_id, states, shape):
    """uint8 [len(states), *shape] frames of the given state indices."""
    states = np.asarray(states, dtype=np.int64)
    fb = int(np.prod(shape))
    assert fb % 4 == 0
    words = fb // 4
    out = frame_hash(scene_id, states[:, None], np.arange(words, dtype=np.uint32)[None, :])
    return out.astype("<u4").view(np.uint8).reshape((len(states),) + tuple(shape))
