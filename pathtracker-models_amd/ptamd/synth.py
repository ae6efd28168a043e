"""Seeded synthetic PathTracker clips (no dataset access on the build or GPU boxes).

Shape and encoding follow the reference's TFRecord payload
(``utils/TFRDataset.py:7-20``): ``image`` = T x 32 x 32 x 3 uint8 frames,
``label`` = ONE raw byte (0x00 / 0x01) that ``engine.prepare_data`` turns into
a float with ``ord()`` (``utils/engine.py:224``).

Content imitates the task: a mostly black frame with a few
saturated distractor dots (red channel) on smooth random walks, one target
dot, a start marker and a goal marker.  The target marker lives in the BLUE
channel of frame 0, because the reference readout reads ``x[:, 2, 0]``
(``models/InT.py:236``).  Values only matter for parity, never for timing.
"""
from __future__ import annotations

import numpy as np


def _walk(rng, t_len, h, w, speed=1.0):
    pos = np.empty((t_len, 2))
    pos[0] = rng.uniform(2, [h - 3, w - 3])
    ang = rng.uniform(0, 2 * np.pi)
    for t in range(1, t_len):
        ang += rng.normal(0.0, 0.35)
        step = speed * np.array([np.sin(ang), np.cos(ang)])
        nxt = pos[t - 1] + step
        for d, lim in enumerate((h, w)):          # reflect off the borders
            if nxt[d] < 1 or nxt[d] > lim - 2:
                step[d] = -step[d]
                ang = np.arctan2(step[0], step[1])
                nxt[d] = pos[t - 1][d] + step[d]
        pos[t] = nxt
    return np.rint(pos).astype(np.int64)


def _dot(frame, y, x, color, r=1):
    h, w, _ = frame.shape
    frame[max(0, y - r):min(h, y + r + 1), max(0, x - r):min(w, x + r + 1)] = color


def make_clip(rng: np.random.Generator, t_len: int = 64, h: int = 32, w: int = 32,
              n_distractors: int = 14, speed: float = 1.0):
    """One clip ``uint8 [T, H, W, 3]`` and its label (0/1)."""
    clip = np.zeros((t_len, h, w, 3), dtype=np.uint8)
    label = int(rng.integers(0, 2))
    tracks = [_walk(rng, t_len, h, w, speed) for _ in range(n_distractors + 1)]
    target = tracks[0]
    # goal marker: where the target ends (positive) or somewhere else (negative)
    if label:
        goal = target[-1]
    else:
        goal = tracks[1][-1] if n_distractors else rng.integers(2, [h - 3, w - 3])
    for t in range(t_len):
        frame = clip[t]
        _dot(frame, int(goal[0]), int(goal[1]), (0, 255, 0), r=2)          # goal (green)
        for tr in tracks[1:]:
            _dot(frame, int(tr[t][0]), int(tr[t][1]), (255, 0, 0))         # distractors
        _dot(frame, int(target[t][0]), int(target[t][1]), (255, 0, 0))   # target
    # start marker of the target, blue channel of frame 0 (read by the readout)
    _dot(clip[0], int(target[0][0]), int(target[0][1]), (0, 0, 255), r=2)
    return clip, label


def make_batch(seed: int, batch: int, t_len: int = 64, h: int = 32, w: int = 32,
               n_distractors: int = 14, speed: float = 1.0):
    """``(uint8 [B, T, H, W, 3], labels)`` seeded by ``seed``.

    Labels are a numpy object array of one-byte ``bytes`` — what a TF string
    tensor's ``.numpy()`` yields — so ``np.vectorize(ord)`` works on it exactly
    as in ``utils/engine.py:224`` (a fixed-width 'S1' array would strip 0x00).
    """
    rng = np.random.default_rng(seed)
    clips = np.empty((batch, t_len, h, w, 3), dtype=np.uint8)
    labels = np.empty((batch,), dtype=object)
    for i in range(batch):
        clips[i], lab = make_clip(rng, t_len, h, w, n_distractors, speed)
        labels[i] = bytes([lab])
    return clips, labels
