"""Deterministic synthetic point clouds: no datasets offline.

splitmix64(seed) -> u in [0,1) as (z >> 40) * 2^-24 (exact fp32). Shapes follow
the reference's loaders: ModelNet40/ShapeNetPart clouds are (B,N,3) in a unit
cube (fed to the model as a permute(0,2,1) view, main_cls.py:91); S3DIS blocks
are (B,N,9) = [xy - 0.5, 3z, rgb, normalised xyz] (prepare_data/indoor3d_util.py:251-260).
"""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(seed, n):
    """n uint64 outputs of splitmix64 started at `seed`."""
    with np.errstate(over="ignore"):
        state = np.uint64(seed) + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = state
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed, shape):
    n = int(np.prod(shape))
    u = (splitmix64(seed, n) >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
    return u.reshape(shape)


def cube_clouds(B, N, seed=0):
    """(B,N,3) float32 in [-1,1): the cls/partseg workload."""
    return (uniform(seed, (B, N, 3)) * np.float32(2.0) - np.float32(1.0)).astype(np.float32)


def tie_clouds(B, N, seed=1, frac=0.01):
    """cube clouds with `frac` of the points duplicated (exact distance ties)."""
    x = cube_clouds(B, N, seed)
    nd = max(1, int(N * frac))
    src = (splitmix64(seed + 7, B * nd) % np.uint64(N)).astype(np.int64).reshape(B, nd)
    dst = (splitmix64(seed + 11, B * nd) % np.uint64(N)).astype(np.int64).reshape(B, nd)
    for b in range(B):
        x[b, dst[b]] = x[b, src[b]]
    return x


def s3dis_blocks(B, N=4096, seed=2):
    """(B,N,9): xy in [-0.5,0.5), z in [0,3), rgb in [0,1), normalised xyz in [0,1)."""
    u = uniform(seed, (B, N, 9))
    u[..., 0:2] -= np.float32(0.5)
    u[..., 2] *= np.float32(3.0)
    return u.astype(np.float32)


def relu_normal(seed, shape):
    """max(0, N(0,1)) features via Box-Muller on the same stream (feature-space kNN)."""
    n = int(np.prod(shape))
    u = uniform(seed, (2, (n + 1) // 1)).astype(np.float64)
    u1 = np.maximum(u[0, :n], 2.0 ** -24)
    g = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u[1, :n])
    return np.maximum(g, 0.0).astype(np.float32).reshape(shape)
