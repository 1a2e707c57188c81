"""Datasets of the reference's ``data`` module (data.py:258-386) with the same
class names, constructor arguments, item layouts and attributes
(``partseg_colors`` / ``semseg_colors`` that main_partseg.py:164 /
main_semseg.py:301 read), so main_cls.py / main_partseg*.py / main_semseg.py
build their loaders unchanged.

Files: the reference's prepared files under ``data/`` (or ``$DGX_DATA_DIR``)
are read when present — h5 layouts of data.py:80-170 via h5py
(modelnet40_ply_hdf5_2048/*.h5, shapenet_part_seg_hdf5_data/*.h5,
indoor3d_sem_seg_hdf5_data[_test]/all_files.txt + room_filelist.txt) and
shapenetpart_<partition>_dataset.pt (data.py:348). A file that exists but cannot
be read raises with the file and the reason. Without files (no network here,
SURVEY §0.6) a dataset serves SYNTHETIC items only when the user opts in with
``DGX_SYNTHETIC_DATA=1`` (a warning says so; ``SYNTHETIC`` records it): items
of the same shapes and dtypes from the repo's splitmix64 stream (dgx.synth),
deterministic and lazy, labels item-derived — plumbing, not learnable data.

Augmentations (data.py:258-276) are restated on numpy arrays: the reference
applies torch ops to numpy items and crashes, here they accept
either and return the input's type.
"""
import glob
import math
import os
import random
import warnings

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

# Visualisation palettes: RGB per part label (50, ShapeNetPart) and per semantic
# class (13, S3DIS) as the reference's prepare_data/meta/{partseg,semseg}_colors.txt
# list them; load_color_partseg / load_color_semseg return these arrays
# (data.py:173-255; the legend PNG they also draw needs cv2 and is not written).
PARTSEG_COLORS = np.array([
    (152, 223, 138), (174, 199, 232), (255, 105, 180), (31, 119, 180), (255, 187, 120), (188, 189, 34),
    (140, 86, 75), (255, 152, 150), (214, 39, 40), (197, 176, 213), (148, 103, 189), (196, 156, 148),
    (23, 190, 207), (186, 85, 211), (247, 182, 210), (66, 188, 102), (219, 219, 141), (140, 57, 197),
    (202, 185, 52), (213, 92, 176), (200, 54, 131), (92, 193, 61), (78, 71, 183), (172, 114, 82),
    (255, 127, 14), (91, 163, 138), (153, 98, 156), (140, 153, 101), (158, 218, 229), (100, 125, 154),
    (178, 127, 135), (120, 185, 128), (146, 111, 194), (44, 160, 44), (112, 128, 144), (96, 207, 209),
    (227, 119, 194), (51, 176, 203), (94, 106, 211), (82, 84, 163), (100, 85, 144), (255, 127, 80),
    (0, 100, 0), (173, 255, 47), (64, 224, 208), (0, 255, 255), (25, 25, 112), (178, 76, 76), (255, 0, 255),
    (152, 223, 138)])
SEMSEG_COLORS = np.array([
    (152, 223, 138), (174, 199, 232), (255, 127, 14), (91, 163, 138), (255, 187, 120), (188, 189, 34),
    (140, 86, 75), (255, 152, 150), (214, 39, 40), (197, 176, 213), (196, 156, 148), (23, 190, 207),
    (112, 128, 144)])


def load_color_partseg():
    """(50, 3) RGB palette of the part labels (reference data.py:173-216)."""
    return PARTSEG_COLORS.copy()


def load_color_semseg():
    """(13, 3) RGB palette of the S3DIS classes (reference data.py:219-255)."""
    return SEMSEG_COLORS.copy()


def synthetic_allowed():
    return os.environ.get("DGX_SYNTHETIC_DATA", "0") == "1"


def _no_files(name, what):
    """No data files: raise, unless the user opted in to synthetic items."""
    if not synthetic_allowed():
        raise FileNotFoundError(
            f"{name}: {what} not found under {os.path.abspath(DATA_DIR)} (set DGX_DATA_DIR to the reference's data "
            "directory; the reference downloads it, data.py:31-77, this build has no network). Set "
            "DGX_SYNTHETIC_DATA=1 to run on synthetic plumbing items instead.")
    warnings.warn(f"{name}: serving SYNTHETIC items ({what} not found, DGX_SYNTHETIC_DATA=1): shapes and dtypes of "
                  "the real dataset, item-derived labels — not learnable data", stacklevel=3)


def _h5_files(pattern):
    files = sorted(glob.glob(os.path.join(DATA_DIR, pattern)))
    if files and h5py is None:
        raise ImportError(f"{files[0]}: reading the reference's h5 files needs h5py, which is not importable")
    return files


def _h5_arrays(files, keys):
    if not files:
        return None
    out = {k: [] for k in keys}
    for f in files:
        try:
            with h5py.File(f, "r") as h:
                for k in keys:
                    out[k].append(h[k][:])
        except (OSError, KeyError) as e:
            raise RuntimeError(f"{f}: cannot read datasets {keys}: {e}") from e
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
        arr = _h5_arrays(_h5_files(f"modelnet40*hdf5_2048/*{partition}*.h5"), ("data", "label"))
        self.SYNTHETIC = arr is None
        if self.SYNTHETIC:
            _no_files("ModelNet40", f"modelnet40_ply_hdf5_2048/*{partition}*.h5")
        else:
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
        arrs = [_h5_arrays(_h5_files(f"shapenet_part_seg_hdf5_data/*{p}*.h5"), ("data", "label", "pid"))
                for p in parts]
        self.SYNTHETIC = any(a is None for a in arrs)
        self.partseg_colors = load_color_partseg()
        if self.SYNTHETIC:
            _no_files("ShapeNetPart", f"shapenet_part_seg_hdf5_data/*{partition}*.h5")
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
    random order for training (data.py:339-364), from the reference's
    data/shapenetpart_<partition>_dataset.pt (data.py:348).

    That file is a pickled ``TensorDataset``, which the safe loader
    (``weights_only=True``) refuses: loading it executes code from the file, so
    it is done only when the user vouches for the file with
    ``DGX_TRUST_PICKLE=1``; a file saved as a tuple / list / dict of the three
    tensors (``torch.save(ds.tensors, path)``) loads safely. Otherwise the
    error names the file and the reason."""

    def __init__(self, partition):
        assert partition in ("train", "trainval", "test")
        self.partition = "train" if partition == "trainval" else partition
        path = os.path.join(DATA_DIR, f"shapenetpart_{self.partition}_dataset.pt")
        self.data = None
        if os.path.exists(path):
            self.data = self._load(path)
        self.SYNTHETIC = self.data is None
        if self.SYNTHETIC:
            _no_files("ShapeNetPart_Augmented", path)
            self.data = ShapeNetPart(2048, self.partition)

    @staticmethod
    def _load(path):
        try:
            obj = torch.load(path, weights_only=True)
        except Exception as e:
            if os.environ.get("DGX_TRUST_PICKLE", "0") != "1":
                raise RuntimeError(
                    f"{path}: the safe loader (torch.load weights_only=True) refuses this file ({type(e).__name__}); "
                    "it is a pickled object (the reference saves a TensorDataset). Re-save it as "
                    "torch.save(ds.tensors, path), or set DGX_TRUST_PICKLE=1 if you trust the file") from e
            obj = torch.load(path, weights_only=False)
        if isinstance(obj, dict):
            obj = tuple(obj[k] for k in ("data", "label", "seg"))
        if isinstance(obj, (tuple, list)):
            obj = torch.utils.data.TensorDataset(*obj)
        return obj

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
    int64 semantic labels in [0, 13) (data.py:367-386); blocks of the test area
    for partition "test", the other areas' otherwise (load_data_semseg,
    data.py:131-170)."""

    def __init__(self, num_points=4096, partition="train", test_area="1"):
        self.num_points = num_points
        self.partition = partition
        self.test_area = str(test_area)
        self.semseg_colors = load_color_semseg()
        sub = "indoor3d_sem_seg_hdf5_data" if partition == "train" else "indoor3d_sem_seg_hdf5_data_test"
        listing = os.path.join(DATA_DIR, sub, "all_files.txt")
        rooms = os.path.join(DATA_DIR, sub, "room_filelist.txt")
        self.SYNTHETIC = not os.path.exists(listing)
        if self.SYNTHETIC:
            _no_files("S3DIS", listing)
            self.n = _SIZES["s3dis"]["train" if partition == "train" else "test"]
            return
        with open(listing) as f:
            files = [os.path.join(DATA_DIR, ln.rstrip()) for ln in f if ln.strip()]
        with open(rooms) as f:
            room_names = [ln.rstrip() for ln in f]
        if h5py is None:
            raise ImportError(f"{listing}: reading the reference's S3DIS h5 blocks needs h5py, which is not importable")
        arr = _h5_arrays(files, ("data", "label"))
        area = "Area_" + self.test_area
        keep = [i for i, r in enumerate(room_names) if (area in r) == (partition != "train")]
        self.data, self.seg = arr["data"][keep], arr["label"][keep]
        self.n = self.data.shape[0]

    def __getitem__(self, item):
        if self.SYNTHETIC:
            block = synth.s3dis_blocks(1, 4096, seed=3000003 + item)[0][:self.num_points]
            seg = (np.arange(self.num_points) * 7 + item) % 13
        else:
            block, seg = self.data[item][:self.num_points], self.seg[item][:self.num_points]
        if self.partition == "train":
            perm = np.random.permutation(block.shape[0])
            block, seg = block[perm], seg[perm]
        return block.astype(np.float32), torch.LongTensor(np.asarray(seg, np.int64))

    def __len__(self):
        return self.n
