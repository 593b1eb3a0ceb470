"""ctypes access to the plain-C oracle (TEST INFRASTRUCTURE ONLY)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_build", "libsdoracle.so")
_P = ctypes.c_void_p


def build():
    src = os.path.join(_HERE, "c", "sd_oracle.c")
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(src):
        return LIB
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB


def _lib():
    build()
    lib = ctypes.CDLL(LIB)
    lib.sdo_gen_rays.argtypes = [_P, _P, _P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                 ctypes.c_float, ctypes.c_float, _P]
    lib.sdo_sample_z.argtypes = [_P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                 _P, _P]
    lib.sdo_voxel_points.argtypes = [_P, ctypes.c_double, ctypes.c_int64, ctypes.c_int64,
                                     ctypes.c_int64, _P, _P]
    return lib


def _p(a):
    return a.ctypes.data_as(_P)


def gen_rays(poses_c2w, Ks, H, W, z_near=3.0, z_far=80.0, frame_ids=None):
    poses_c2w = np.ascontiguousarray(poses_c2w, np.float32)
    Ks = np.ascontiguousarray(Ks, np.float32)
    v = poses_c2w.shape[0]
    ids = np.arange(v, dtype=np.float32) if frame_ids is None else np.ascontiguousarray(frame_ids, np.float32)
    out = np.empty((v, H, W, 11), np.float32)
    _lib().sdo_gen_rays(_p(poses_c2w), _p(Ks), _p(ids), v, H, W, z_near, z_far, _p(out))
    return out


def sample_z(rays, K, u, lindisp=True):
    rays = np.ascontiguousarray(rays, np.float32)
    u = np.ascontiguousarray(u, np.float32)
    R, rd = rays.shape
    z = np.empty((R, K), np.float32)
    _lib().sdo_sample_z(_p(rays), R, rd, K, int(lindisp), _p(u), _p(z))
    return z


def voxel_points(origin, vox, dims, T):
    origin = np.ascontiguousarray(origin, np.float64)
    T = np.ascontiguousarray(T, np.float64)
    nx, ny, nz = dims
    out = np.empty((nx * ny * nz, 3), np.float32)
    _lib().sdo_voxel_points(_p(origin), float(vox), nx, ny, nz, _p(T), _p(out))
    return out
