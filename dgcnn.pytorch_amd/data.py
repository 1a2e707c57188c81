"""Datasets of the reference's ``data`` module (data.py:258-386) with the same
class names, constructor arguments and item layouts, so main_cls.py /
main_partseg*.py / main_semseg.py build their loaders unchanged.

Files: when h5py is importable and the reference's h5 files are present under
``data/`` (data.py:80-170 layouts: modelnet40_ply_hdf5_2048/ply_data_*.h5,
shapenet_part_seg_hdf5_data/*.h5, indoor3d_sem_seg_hdf5_data_test/ ...), they
are read. Otherwise (no network, no h5py in this image: SURVEY §0.6) every
dataset serves SYNTHETIC items of the same shapes and dtypes, generated per
item from the repo's splitmix64 stream (dgx.synth), deterministic and lazy (no
dataset-sized arrays in memory): labels are item-derived, so they are
plumbing, not learnable data. ``SYNTHETIC`` records which one a dataset uses.

Augmentations (data.py:258-276) are restated on numpy arrays: the reference
applies torch ops to numpy items and crashes, here they accept
either and return the input's type.
"""
import glob
import math
import os
import random

import numpy as np
import torch
from torch.utils.data import Dataset

from dgx import synth

try:  # optional: only to read the reference's real files when they exist
    import h5py
except ImportError:  # not in this image
    h5py = None

DATA_DIR = os.environ.get("DGX_DATA_DIR", "data")
# split sizes of the real datasets (used for the synthetic stand-ins)
_SIZES = {"modelnet40": {"train": 9840, "test": 2468},
          "shapenetpart": {"train": 12137, "trainval": 14007, "val": 1870, "test": 2874},
          "s3dis": {"train": 20291, "test": 3294}}


def _h5_arrays(pattern, keys):
    files = sorted(glob.glob(os.path.join(DATA_DIR, pattern)))
    if h5py is None or not files:
        return None
    out = {k: [] for k in keys}
    for f in files:
        with h5py.File(f, "r") as h:
            for k in keys:
                out[k].append(h[k][:])
    return {k: np.concatenate(v, axis=0) for k, v in out.items()}


def _synthetic_cloud(seed, n, channels=3):
    """(n, channels) float32 cloud in [-1, 1) from the item's seed."""
    return (2.0 * synth.uniform(seed, (n, channels)) - 1.0).astype(np.float32)


def _as_numpy(pc):
    return pc.numpy() if isinstance(pc, torch.Tensor) else pc


def _like(out, ref):
    return torch.from_numpy(out) if isinstance(ref, torch.Tensor) else out


def translate_pointcloud(pointcloud):
    """Scale each axis by U(2/3, 3/2) and shift by U(-0.2, 0.2) (data.py:258-262)."""
    pc = _as_numpy(pointcloud)
    scale = np.random.uniform(2.0 / 3.0, 3.0 / 2.0, size=3).astype(np.float32)
    shift = np.random.uniform(-0.2, 0.2, size=3).astype(np.float32)
    return _like((pc * scale + shift).astype(np.float32), pointcloud)


def jitter_pointcloud(pointcloud, sigma=0.01, clip=0.02):
    """Add clipped Gaussian noise (data.py:265-268)."""
    pc = _as_numpy(pointcloud)
    noise = np.clip(sigma * np.random.randn(*pc.shape), -clip, clip).astype(np.float32)
    return _like(pc + noise, pointcloud)


def rotate_pointcloud(pointcloud):
    """Random rotation in the x-z plane (data.py:271-276)."""
    pc = _as_numpy(pointcloud).copy()
    theta = 2.0 * math.pi * np.random.randn()
    rot = np.array([[math.cos(theta), -math.sin(theta)], [math.sin(theta), math.cos(theta)]], np.float32)
    pc[:, [0, 2]] = pc[:, [0, 2]] @ rot
    return _like(pc, pointcloud)


class ModelNet40(Dataset):
    """(num_points, 3) float32 cloud, (1,) int64 label in [0, 40) (data.py:279-294)."""

    def __init__(self, num_points, partition="train"):
        self.num_points = num_points
        self.partition = partition
        arr = _h5_arrays(f"modelnet40*hdf5_2048/*{partition}*.h5", ("data", "label"))
        self.SYNTHETIC = arr is None
        if arr is not None:
            self.data, self.label = arr["data"].astype(np.float32), arr["label"].astype(np.int64)
        self.n = _SIZES["modelnet40"][partition] if self.SYNTHETIC else self.data.shape[0]

    def __getitem__(self, item):
        if self.SYNTHETIC:
            pc = _synthetic_cloud(1000003 * (1 + (self.partition == "test")) + item, 2048)[:self.num_points]
            label = np.array([item % 40], np.int64)
        else:
            pc, label = self.data[item][:self.num_points], self.label[item]
        if self.partition == "train":
            pc = translate_pointcloud(pc)
            np.random.shuffle(pc)
        return pc, label

    def __len__(self):
        return self.n


class ShapeNetPart(Dataset):
    """(num_points, 3) cloud, (1,) category, (num_points,) part labels (data.py:297-336)."""
    cat2id = {"airplane": 0, "bag": 1, "cap": 2, "car": 3, "chair": 4, "earphone": 5, "guitar": 6, "knife": 7,
              "lamp": 8, "laptop": 9, "motor": 10, "mug": 11, "pistol": 12, "rocket": 13, "skateboard": 14,
              "table": 15}
    seg_num = [4, 2, 2, 4, 4, 3, 3, 2, 4, 2, 6, 2, 3, 3, 3, 3]
    index_start = [0, 4, 6, 8, 12, 16, 19, 22, 24, 28, 30, 36, 38, 41, 44, 47]

    def __init__(self, num_points, partition="train", class_choice=None):
        self.num_points = num_points
        self.partition = partition
        self.class_choice = class_choice
        parts = ("train", "val") if partition == "trainval" else (partition,)
        arrs = [_h5_arrays(f"shapenet_part_seg_hdf5_data/*{p}*.h5", ("data", "label", "pid")) for p in parts]
        self.SYNTHETIC = any(a is None for a in arrs)
        if self.SYNTHETIC:
            n = _SIZES["shapenetpart"][partition]
            self.labels = np.arange(n, dtype=np.int64) % 16
        else:
            self.data = np.concatenate([a["data"] for a in arrs]).astype(np.float32)
            self.labels = np.concatenate([a["label"] for a in arrs]).astype(np.int64).reshape(-1)
            self.seg = np.concatenate([a["pid"] for a in arrs]).astype(np.int64)
        self.items = np.arange(len(self.labels))
        if class_choice is not None:
            cid = self.cat2id[class_choice]
            self.items = self.items[self.labels == cid]
            self.seg_num_all, self.seg_start_index = self.seg_num[cid], self.index_start[cid]
        else:
            self.seg_num_all, self.seg_start_index = 50, 0

    def __getitem__(self, item):
        i = int(self.items[item])
        cat = int(self.labels[i])
        if self.SYNTHETIC:
            pc = _synthetic_cloud(2000003 + i, 2048)[:self.num_points]
            seg = (self.index_start[cat] + np.arange(self.num_points) % self.seg_num[cat]).astype(np.int64)
        else:
            pc, seg = self.data[i][:self.num_points], self.seg[i][:self.num_points]
        if self.partition == "trainval":
            perm = np.random.permutation(pc.shape[0])
            pc, seg = pc[perm], seg[perm]
        return pc, np.array([cat], np.int64), seg

    def __len__(self):
        return len(self.items)


class ShapeNetPart_Augmented(Dataset):
    """(pointcloud, label, seg) tensors with random translate / jitter / rotate in
    random order for training (data.py:339-364). Reads the reference's
    data/shapenetpart_<partition>_dataset.pt (a saved TensorDataset) with the
    safe loader when present, else synthetic ShapeNetPart items (2048 points)."""

    def __init__(self, partition):
        assert partition in ("train", "trainval", "test")
        self.partition = "train" if partition == "trainval" else partition
        path = os.path.join(DATA_DIR, f"shapenetpart_{self.partition}_dataset.pt")
        self.data = None
        if os.path.exists(path):
            try:
                self.data = torch.load(path, weights_only=True)
            except Exception:  # a pickled TensorDataset: refused by the safe loader
                self.data = None
        self.SYNTHETIC = self.data is None
        if self.SYNTHETIC:
            self.data = ShapeNetPart(2048, self.partition)

    def __len__(self):
        return len(self.data)

    def __getitem__(self, index):
        pc, label, seg = self.data[index]
        pc, label, seg = (torch.as_tensor(np.asarray(v)) if not isinstance(v, torch.Tensor) else v
                          for v in (pc, label, seg))
        if self.partition == "train":
            fns = [translate_pointcloud, jitter_pointcloud, rotate_pointcloud]
            random.shuffle(fns)
            for fn, on in zip(fns, torch.randint(0, 2, (3,)).tolist()):
                if on:
                    pc = fn(pc)
        return pc, label, seg


class S3DIS(Dataset):
    """(num_points, 9) block [xy - c, z, rgb, normalised xyz] and (num_points,)
    int64 semantic labels in [0, 13) (data.py:367-386)."""

    def __init__(self, num_points=4096, partition="train", test_area="1"):
        self.num_points = num_points
        self.partition = partition
        self.test_area = str(test_area)
        self.SYNTHETIC = True  # the reference's prepared S3DIS h5 is not readable here (no h5py)
        self.n = _SIZES["s3dis"]["train" if partition == "train" else "test"]

    def __getitem__(self, item):
        block = synth.s3dis_blocks(1, 4096, seed=3000003 + item)[0][:self.num_points]
        seg = (np.arange(self.num_points) * 7 + item) % 13
        if self.partition == "train":
            perm = np.random.permutation(block.shape[0])
            block, seg = block[perm], seg[perm]
        return block.astype(np.float32), torch.LongTensor(seg)

    def __len__(self):
        return self.n
