"""Load step's keyframe detection (btnLoadClick main.pas:984-1166) on libANN.so.

Frames are what FrameTiling takes: [F][tm_h*tm_w][64] int32 0x00BBGGRR tiles (TFrame.Tiles, LoadFrame
main.pas:3211-3266).  Decoding image files / ffmpeg (DoExternalFFMpeg) stays out of scope: the caller
hands over frames already in memory.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, load

TILE_MAP_MAX_W, TILE_MAP_MAX_H = 1920 // 8, 1080 // 8  # ReframeUI main.pas:1933-1934 (the reference's cap)


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def interframe_correlation(frames, tm_w: int, tm_h: int) -> np.ndarray:
    """corr[i-1] = ComputeInterFrameCorrelation(frame i-1, frame i) (main.pas:811-828), host arrays."""
    frames = np.ascontiguousarray(frames, np.int32).reshape(-1, tm_w * tm_h * 64)
    F = frames.shape[0]
    corr = np.zeros(max(0, F - 1), np.float64)
    check(load().tiler_interframe_correlation(_p(frames), F, tm_w, tm_h, _p(corr)), "tiler_interframe_correlation")
    return corr


def interframe_correlation_dev(d_rgb: int, F: int, tm_w: int, tm_h: int, stream=None) -> np.ndarray:
    """Same with the frames resident in HBM (device pointer), synchronous on `stream`."""
    corr = np.zeros(max(0, F - 1), np.float64)
    check(load().tiler_interframe_correlation_dev(ctypes.c_void_p(d_rgb), F, tm_w, tm_h, _p(corr),
                                                  ctypes.c_void_p(stream) if stream else None),
          "tiler_interframe_correlation_dev")
    return corr


def find_keyframes(corr, F: int, tile_map_size: int):
    """The shot-transition split (main.pas:1099-1132): (keyframe index per frame, keyframe count)."""
    corr = np.ascontiguousarray(corr, np.float64)
    if corr.size < max(0, F - 1):
        raise ValueError("find_keyframes: need F-1 correlations")
    kf = np.zeros(F, np.int32)
    n = check(load().tiler_find_keyframes(_p(corr), F, tile_map_size, _p(kf)), "tiler_find_keyframes")
    return kf, n


def keyframe_starts(kf_of_frame) -> np.ndarray:
    """FKeyFrames[j].StartFrame (main.pas:1136-1146) as kf_start[KF+1] (the encoder's Video.kf_start)."""
    kf = np.asarray(kf_of_frame, np.int64)
    if kf.size == 0:
        return np.zeros(1, np.int64)
    starts = np.flatnonzero(np.r_[True, kf[1:] != kf[:-1]])
    return np.r_[starts, kf.size].astype(np.int64)


def detect_keyframes(frames, tm_w: int, tm_h: int):
    """btnLoadClick's keyframe pass: correlations on the GPU, split on the host -> (kf_of_frame, kf_start, corr)."""
    frames = np.ascontiguousarray(frames, np.int32).reshape(-1, tm_w * tm_h * 64)
    F = frames.shape[0]
    corr = interframe_correlation(frames, tm_w, tm_h)
    kf, _ = find_keyframes(corr, F, tm_w * tm_h)
    return kf, keyframe_starts(kf), corr
