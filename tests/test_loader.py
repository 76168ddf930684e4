"""Data path: the HBM-resident loader and the inference export vs the
restated reference collators (oracle/collate_ref.py: src/dataloader.py:21-121,
src/Prediction.py:21-52,115-126) on synthetic MicroLens-shaped parquet files.

CPU tests: parquet reading, the item_info index, error rules, checkpoint interop, CSV/zip export.
GPU tests (-m gpu): every batch of the device collator bit-identical to the reference collator's.
"""
import os
import zipfile

import numpy as np
import pytest
import torch

from ctr_recommendation_amd.data import write_microlens_parquet
from ctr_recommendation_amd.loader import ColumnarDataset, DeviceLoader, ItemInfoTable, read_parquet_columns
from oracle.collate_ref import BatchCollatorRef, InferenceCollatorRef, batches, export_submission, load_data


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("microlens")
    # item_seq stored 25 wide (> max_len 20: the truncation path); non-contiguous ids (stride 3)
    return write_microlens_parquet(str(d), n_train=1000, n_valid=300, n_test=700, n_items=400, seq_width=25,
                                   item_id_stride=3, seed=7)


@pytest.fixture(scope="module")
def files_missing(tmp_path_factory):
    d = tmp_path_factory.mktemp("microlens_missing")
    # item 1 + 3*5 = 16 has no item_info row
    return write_microlens_parquet(str(d), n_train=600, n_test=600, n_items=50, seq_width=20, item_id_stride=3,
                                   missing_ids=[16], seed=11)


# ---------------------------------------------------------------- CPU
def test_columns_match_reference_column_stack(files):
    darray, ci = load_data(files["train_data"])
    cols = read_parquet_columns(files["train_data"])
    for name, idx in ci.items():
        ref = darray[:, idx]
        got = cols[name].astype(np.float64)
        assert np.array_equal(ref, got if got.ndim == ref.ndim else got.reshape(ref.shape)), name


def test_item_info_index_and_errors(files):
    cols = read_parquet_columns(files["item_info"])
    info = ItemInfoTable(cols["item_id"], cols["item_emb_d128"], "cpu")
    slot = info.slot_of_id.numpy()
    assert info.n_ids == int(cols["item_id"].max()) + 1
    assert (slot[cols["item_id"]] == np.arange(len(cols["item_id"]))).all()
    assert (np.delete(slot, cols["item_id"]) == -1).all()                # ids 0, 2, 3, 5, ... absent
    with pytest.raises(ValueError):
        ItemInfoTable(np.array([1, 1]), np.zeros((2, 128), np.float32), "cpu")


def test_ragged_list_column_raises(tmp_path):
    import pyarrow as pa
    import pyarrow.parquet as pq
    p = str(tmp_path / "ragged.parquet")
    pq.write_table(pa.table({"item_id": pa.array([1, 2]), "item_seq": pa.array([[1, 2], [3]])}), p)
    with pytest.raises(ValueError):
        read_parquet_columns(p)


def test_reference_collator_restatement(files, files_missing):
    """The oracle collators on hand-checkable facts: the last 20 of 25 history slots, ids as
    int64 after the model's casts, the item_info row of each id, KeyError on an unknown id (train),
    the whole-batch zero fallback (inference)."""
    darray, ci = load_data(files["train_data"])
    col = BatchCollatorRef(20, ci, files["item_info"])
    b, y = next(batches(darray, col, 64))
    assert b["item_seq"].shape == (64, 20)
    assert torch.equal(b["item_seq"], torch.from_numpy(darray[:64, ci["item_seq"][-20:]]).long())
    assert torch.equal(y, torch.from_numpy(darray[:64, ci["label"]]).float())
    info = read_parquet_columns(files["item_info"])
    row = np.searchsorted(info["item_id"], darray[:64, ci["item_id"]].astype(np.int64))
    assert torch.equal(b["item_emb_d128"], torch.from_numpy(info["item_emb_d128"][row]))
    dm, cim = load_data(files_missing["train_data"])
    colm = BatchCollatorRef(20, cim, files_missing["item_info"])
    with pytest.raises(KeyError):
        for _ in batches(dm, colm, 64):
            pass
    dt, cit = load_data(files_missing["test_data"])
    inf = InferenceCollatorRef(20, cit, files_missing["item_info"])
    for bt in batches(dt, inf, 64):
        has_missing = (bt["item_id"].numpy() == 16).any()
        assert bool((bt["item_emb_d128"] == 0).all()) == bool(has_missing)


def test_reference_collator_breaks_on_a_one_row_batch(files):
    """A final batch of ONE row (1000 rows at batch 333): the reference's ``squeeze(-1)``
    (src/dataloader.py:80) makes the ids 0-d, ``.loc`` then returns a Series and
    ``.values`` fails (:94).  The device loader returns the row as a batch of one instead (shapes
    (1,), (1, 20), (1, 128)); this is the one place it does not reproduce the reference."""
    darray, ci = load_data(files["train_data"])
    with pytest.raises(AttributeError):
        list(batches(darray, BatchCollatorRef(20, ci, files["item_info"]), 333))


def test_checkpoint_interop_module_prefix(tmp_path):
    """A DataParallel checkpoint (``module.`` keys, src/train_fibinet.py:150 saves without them,
    Prediction.py strips them) loads strictly into the drop-in module."""
    from ctr_recommendation_amd.model_fibinet import build_model
    from ctr_recommendation_amd.predict import load_checkpoint
    from oracle.fibinet_oracle import build_model as oracle_build
    cfg = {"embedding_dim": 16, "vocab_size": 500}
    torch.manual_seed(3)
    ref = oracle_build(None, cfg)
    p = str(tmp_path / "FiBiNET_best.pth")
    torch.save({"module." + k: v for k, v in ref.state_dict().items()}, p)
    m = build_model(None, cfg)
    m.load_state_dict(load_checkpoint(p))                 # strict
    for k, v in ref.state_dict().items():
        assert torch.equal(m.state_dict()[k], v), k


def test_export_byte_identical(tmp_path):
    from ctr_recommendation_amd.predict import export_submission as ours
    rng = np.random.default_rng(0)
    preds = rng.random(1000).astype(np.float32)
    os.chdir(tmp_path)
    export_submission(preds, "ref.csv", "ref.zip")
    ours(preds, "prediction_fibinet.csv", "submission_fibinet.zip")
    assert open("ref.csv", "rb").read() == open("prediction_fibinet.csv", "rb").read()
    with zipfile.ZipFile("submission_fibinet.zip") as zf:
        assert zf.namelist() == ["prediction_fibinet.csv"]
        assert zf.read("prediction_fibinet.csv") == open("ref.csv", "rb").read()
    head = open("prediction_fibinet.csv").read().splitlines()[:2]
    assert head[0] == "ID,Task2" and head[1].startswith("0,")


# ---------------------------------------------------------------- GPU
def _ours(files, dev, split, mode, bs, **kw):
    info = ItemInfoTable.from_parquet(files["item_info"], dev)
    ds = ColumnarDataset.from_parquet(files[f"{split}_data"], dev)
    return DeviceLoader(ds, info, bs, shuffle=False, max_len=20, mode=mode, **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("bs", [128, 300])
def test_device_collator_matches_reference_train(files, hip_device, bs):
    """Every batch (the last one short) bit-identical to BatchCollator's: ids, truncated history,
    levels, user ids, item_info rows, labels."""
    darray, ci = load_data(files["train_data"])
    ref = list(batches(darray, BatchCollatorRef(20, ci, files["item_info"]), bs))
    ours = _ours(files, hip_device, "train", "train", bs)
    assert len(ours) == len(ref)
    for (rb, ry), (hb, hy) in zip(ref, ours):
        for k in ("item_id", "item_seq", "likes_level", "views_level", "user_id"):
            assert torch.equal(rb[k].long(), hb[k].cpu()), k
            assert hb[k].dtype == torch.int64
        assert torch.equal(rb["item_emb_d128"], hb["item_emb_d128"].cpu())
        assert torch.equal(ry, hy.cpu())
    ours.check()


@pytest.mark.gpu
def test_device_collator_sorted_id_index(files, hip_device, monkeypatch):
    """The sparse-id item_info index (ids sorted, binary search per sample -- what a table of
    hashed ids gets instead of a dense index sized by the largest id): the same batches,
    bit-identical to BatchCollator's."""
    monkeypatch.setattr(ItemInfoTable, "DENSE_FACTOR", 0)
    monkeypatch.setattr(ItemInfoTable, "DENSE_SLACK", 0)
    darray, ci = load_data(files["train_data"])
    ref = list(batches(darray, BatchCollatorRef(20, ci, files["item_info"]), 128))
    ours = _ours(files, hip_device, "train", "train", 128)
    assert ours.info.sorted_ids is not None
    for (rb, ry), (hb, hy) in zip(ref, ours):
        assert torch.equal(rb["item_emb_d128"], hb["item_emb_d128"].cpu())
        assert torch.equal(rb["item_id"].long(), hb["item_id"].cpu())
    ours.check()


def test_item_info_index_choice():
    """Dense id -> row index for compact ids; sorted ids for sparse ones (largest id far beyond
    the row count): the index never scales with the largest id."""
    ids = np.array([3, 1, 7, 2], dtype=np.int64)
    emb = np.arange(16, dtype=np.float32).reshape(4, 4)
    t = ItemInfoTable(ids, emb, "cpu")
    assert t.sorted_ids is None and t.n_ids == 8 and t.slot_of_id[7].item() == 2
    big = np.array([5, 1 << 40, 17, 1 << 33], dtype=np.int64)
    t = ItemInfoTable(big, emb, "cpu")
    assert t.sorted_ids is not None and t.n_ids == 4
    assert t.sorted_ids.tolist() == sorted(big.tolist())
    assert [int(big[k]) for k in t.slot_of_id.tolist()] == sorted(big.tolist())


@pytest.mark.gpu
def test_device_collator_unknown_ids(files_missing, hip_device):
    """Training: the reference's KeyError (raised by check()); inference: the whole batch of an
    unknown id gets zero mm vectors, every other batch its item_info rows."""
    tr = _ours(files_missing, hip_device, "train", "train", 64)
    for _ in tr:
        pass
    with pytest.raises(KeyError):
        tr.check()
    dt, cit = load_data(files_missing["test_data"])
    ref = list(batches(dt, InferenceCollatorRef(20, cit, files_missing["item_info"]), 64))
    ours = list(_ours(files_missing, hip_device, "test", "inference", 64))
    assert len(ours) == len(ref)
    zeroed = 0
    for rb, hb in zip(ref, ours):
        assert torch.equal(rb["item_emb_d128"], hb["item_emb_d128"].cpu())
        assert torch.equal(rb["item_seq"], hb["item_seq"].cpu())
        zeroed += int((rb["item_emb_d128"] == 0).all())
    assert 0 < zeroed < len(ref)


@pytest.mark.gpu
def test_rank_slices_cover_the_global_batch(files, hip_device):
    """rank r of N gets its contiguous share of each global batch (the sharded trainer's input)."""
    full = [b for b, _ in _ours(files, hip_device, "train", "train", 200)]
    parts = [[b for b, _ in _ours(files, hip_device, "train", "train", 200, rank=r, world=4)] for r in range(4)]
    for i, fb in enumerate(full):
        cat = torch.cat([parts[r][i]["item_id"] for r in range(4)])
        assert torch.equal(cat, fb["item_id"])


@pytest.mark.gpu
def test_predict_export_end_to_end(files, hip_device, tmp_path):
    """Prediction.py's flow on the drop-in module: strict load of a module.-prefixed checkpoint,
    eval forward at batch 8192 through the inference loader, CSV + zip; predictions equal the
    oracle's forward over the reference collator's batches (1e-4, the logit bar)."""
    from ctr_recommendation_amd.model_fibinet import build_model
    from ctr_recommendation_amd.predict import export_submission as ours_export
    from ctr_recommendation_amd.predict import load_checkpoint, predict
    from oracle.fibinet_oracle import build_model as oracle_build
    cfg = {"embedding_dim": 16, "vocab_size": 1300}
    torch.manual_seed(5)
    ref = oracle_build(None, cfg).eval()
    p = str(tmp_path / "ck.pth")
    torch.save({"module." + k: v for k, v in ref.state_dict().items()}, p)
    m = build_model(None, cfg)
    m.load_state_dict(load_checkpoint(p))
    m.to(hip_device)
    preds = predict(m, _ours(files, hip_device, "test", "inference", 8192))
    dt, cit = load_data(files["test_data"])
    with torch.no_grad():
        rp = np.concatenate([ref(b).numpy() for b in batches(dt, InferenceCollatorRef(20, cit, files["item_info"]),
                                                              8192)])
    assert preds.shape == rp.shape
    assert np.abs(preds - rp).max() < 1e-4
    os.chdir(tmp_path)
    ours_export(preds)
    assert os.path.exists("submission_fibinet.zip")
