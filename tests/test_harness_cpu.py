"""CPU tests of the script-facing modules the reference imports but does not
ship or cannot run here: util.cal_loss /
IOStream, model.PointNet / DGCNN_cls / DGCNN_semseg (construction, state_dict
names), data.* datasets (synthetic stand-ins: shapes, dtypes, augmentations)."""
import types

import numpy as np
import torch


def test_cal_loss_label_smoothing():
    from util import cal_loss
    torch.manual_seed(0)
    pred = torch.randn(7, 40)
    gold = torch.randint(0, 40, (7,))
    eps = 0.2
    target = torch.full((7, 40), eps / 39)
    target[torch.arange(7), gold] = 1 - eps
    want = -(target * torch.log_softmax(pred, 1)).sum(1).mean()
    assert torch.allclose(cal_loss(pred, gold), want, atol=1e-6)
    assert torch.allclose(cal_loss(pred, gold.view(7, 1), smoothing=False),
                          torch.nn.functional.cross_entropy(pred, gold), atol=1e-6)


def test_iostream(tmp_path):
    from util import IOStream
    io = IOStream(str(tmp_path / "run.log"))
    io.cprint("hello")
    io.close()
    assert (tmp_path / "run.log").read_text() == "hello\n"


def test_models_construct_with_upstream_names():
    from model import DGCNN_cls, DGCNN_semseg, PointNet
    args = types.SimpleNamespace(k=20, emb_dims=1024, dropout=0.5)
    cls = DGCNN_cls(args)
    keys = list(cls.state_dict().keys())
    assert keys[0] == "bn1.weight" and "conv1.0.weight" in keys and "conv5.0.weight" in keys
    assert tuple(cls.conv1[0].weight.shape) == (64, 6, 1, 1) and tuple(cls.conv5[0].weight.shape) == (1024, 512, 1)
    assert tuple(cls.linear3.weight.shape) == (40, 256)
    seg = DGCNN_semseg(args)
    assert tuple(seg.conv1[0].weight.shape) == (64, 18, 1, 1) and tuple(seg.conv7[0].weight.shape) == (512, 1216, 1)
    assert tuple(seg.conv9.weight.shape) == (13, 256, 1)
    pn = PointNet(args)
    pn.eval()
    assert tuple(pn(torch.randn(2, 3, 64)).shape) == (2, 40)  # PointNet is stock torch: runs on CPU


def test_datasets_synthetic_items(monkeypatch, tmp_path):
    import data
    monkeypatch.setattr(data, "DATA_DIR", str(tmp_path))
    monkeypatch.setenv("DGX_SYNTHETIC_DATA", "1")
    mn = data.ModelNet40(1024, "train")
    pc, label = mn[3]
    assert mn.SYNTHETIC and len(mn) == 9840
    assert pc.shape == (1024, 3) and pc.dtype == np.float32 and label.dtype == np.int64 and 0 <= label[0] < 40
    te = data.ModelNet40(1024, "test")
    a, _ = te[5]
    b, _ = te[5]
    assert np.array_equal(a, b)  # test items are deterministic (no augmentation)
    sp = data.ShapeNetPart(2048, "trainval")
    pc, cat, seg = sp[10]
    assert pc.shape == (2048, 3) and seg.shape == (2048,) and seg.dtype == np.int64
    assert sp.seg_start_index == 0 and sp.seg_num_all == 50
    one = data.ShapeNetPart(2048, "test", class_choice="chair")
    pc, cat, seg = one[0]
    assert int(cat[0]) == 4 and seg.min() >= 12 and seg.max() < 16
    aug = data.ShapeNetPart_Augmented("train")
    pc, cat, seg = aug[1]
    assert isinstance(pc, torch.Tensor) and tuple(pc.shape) == (2048, 3)
    s3 = data.S3DIS(4096, "train")
    blk, seg = s3[2]
    assert blk.shape == (4096, 9) and seg.dtype == torch.int64 and int(seg.max()) < 13


def test_augmentations_accept_numpy_and_tensors():
    import data
    np.random.seed(0)
    pc = np.random.rand(100, 3).astype(np.float32)
    for fn in (data.translate_pointcloud, data.jitter_pointcloud, data.rotate_pointcloud):
        out = fn(pc.copy())
        assert isinstance(out, np.ndarray) and out.shape == pc.shape and out.dtype == np.float32
        out_t = fn(torch.from_numpy(pc.copy()))
        assert isinstance(out_t, torch.Tensor) and tuple(out_t.shape) == pc.shape
    # rotation in the x-z plane keeps y and the x-z norms
    r = data.rotate_pointcloud(pc.copy())
    assert np.allclose(r[:, 1], pc[:, 1])
    assert np.allclose(np.hypot(r[:, 0], r[:, 2]), np.hypot(pc[:, 0], pc[:, 2]), atol=1e-5)


def test_datasets_fail_loudly_without_files(monkeypatch, tmp_path):
    """No data files and no opt-in: every dataset raises, naming what is missing
    (the reference would download them, data.py:31-77)."""
    import pytest
    import data
    monkeypatch.setattr(data, "DATA_DIR", str(tmp_path))
    monkeypatch.delenv("DGX_SYNTHETIC_DATA", raising=False)
    for make in (lambda: data.ModelNet40(1024), lambda: data.ShapeNetPart(2048), lambda: data.S3DIS(4096),
                 lambda: data.ShapeNetPart_Augmented("train")):
        with pytest.raises(FileNotFoundError, match="DGX_SYNTHETIC_DATA"):
            make()


def test_augmented_refuses_pickled_dataset(monkeypatch, tmp_path):
    """The reference's shapenetpart_<p>_dataset.pt is a pickled TensorDataset: the
    safe loader refuses it, and the dataset raises naming the file instead of
    silently switching to synthetic items; a tensors-tuple file loads."""
    import pytest
    import data
    monkeypatch.setattr(data, "DATA_DIR", str(tmp_path))
    monkeypatch.delenv("DGX_TRUST_PICKLE", raising=False)
    tensors = (torch.rand(3, 2048, 3), torch.arange(3).view(3, 1), torch.zeros(3, 2048, dtype=torch.int64))
    torch.save(torch.utils.data.TensorDataset(*tensors), tmp_path / "shapenetpart_train_dataset.pt")
    with pytest.raises(RuntimeError, match="shapenetpart_train_dataset.pt"):
        data.ShapeNetPart_Augmented("train")
    torch.save(tensors, tmp_path / "shapenetpart_test_dataset.pt")
    ds = data.ShapeNetPart_Augmented("test")
    assert not ds.SYNTHETIC and len(ds) == 3 and torch.equal(ds[1][0], tensors[0][1])


def test_color_palettes_as_scripts_read_them(monkeypatch, tmp_path):
    """main_partseg.py:164 / main_semseg.py:301 read the datasets' palettes."""
    import data
    monkeypatch.setattr(data, "DATA_DIR", str(tmp_path))
    monkeypatch.setenv("DGX_SYNTHETIC_DATA", "1")
    pc = data.ShapeNetPart(2048, "test").partseg_colors
    sc = data.S3DIS(4096, "test").semseg_colors
    assert pc.shape == (50, 3) and sc.shape == (13, 3)
    assert pc.min() >= 0 and pc.max() <= 255 and tuple(pc[0]) == (152, 223, 138) and tuple(sc[12]) == (112, 128, 144)


def test_bench_pmc_traffic_only_for_preset_shapes():
    """bench.py's roofline `traffic` comes from committed PMC counters of the
    preset's launches; another batch size launches other grids (and, for few
    clouds, another kNN kernel), so the lookup refuses it."""
    import types
    import bench
    args = types.SimpleNamespace(config="cfg2", points=1024, k=20, batch=4)
    traffic, note = bench.pmc_traffic(args, [3, 64, 64, 128], 4)
    assert traffic is None and "no PMC profile for B=4" in note
