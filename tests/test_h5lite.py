"""HDF5 subset: reference fixture decoding and writer round-trips."""
import os

import numpy as np
import pytest

from alphago_amd.io.h5lite import H5File, H5Writer

FIXTURE = "/root/reference/tests/test_data/hdf5/alphago-vs-lee-sedol-features.hdf5"


@pytest.mark.skipif(not os.path.exists(FIXTURE), reason="reference fixture absent")
def test_reads_reference_fixture():
    with H5File(FIXTURE) as f:
        assert sorted(f.keys()) == ["actions", "file_offsets", "states"]
        s, a = f["states"].read(), f["actions"].read()
        assert s.shape == (1033, 12, 19, 19) and s.dtype == np.uint8
        assert a.shape == (1033, 2)
        assert set(np.unique(s)) <= {0, 1}
        # plane 3 of 12 ('ones') is constant 1 (board(3), ones(1), turns_since(8))
        assert s[:, 3].min() == 1
        offs = {k: tuple(f["file_offsets"][k].read()) for k in f["file_offsets"].keys()}
        assert sum(n for _, n in offs.values()) == 1033


def test_writer_roundtrip(tmp_path):
    p = str(tmp_path / "x.h5")
    rng = np.random.default_rng(0)
    w32 = rng.standard_normal((5, 3, 3, 3)).astype(np.float32)
    with H5Writer(p) as f:
        f.attrs["layer_names"] = np.array([b"conv_1", b"flatten_2"])
        f.attrs["scalar"] = 3.5
        g = f.create_group("conv_1")
        g.attrs["weight_names"] = np.array([b"conv_1_W", b"conv_1_b"])
        g["conv_1_W"] = w32
        g["conv_1_b"] = np.arange(5, dtype=np.float32)
        f.create_group("flatten_2").attrs["weight_names"] = np.zeros((0,), dtype="S1")
        s = f.stream_dataset("states", (4, 19, 19), np.uint8)
        blocks = [rng.integers(0, 2, (n, 4, 19, 19), dtype=np.uint8) for n in (3, 7, 1)]
        for b in blocks:
            s.append(b)
        many = f.create_group("file_offsets")
        for i in range(300):  # forces multiple symbol nodes and a 2-level B-tree
            many["game_%04d.sgf" % i] = np.array([i, i + 1], dtype=np.int64)
    with H5File(p) as f:
        assert list(f.attrs["layer_names"]) == [b"conv_1", b"flatten_2"]
        assert f.attrs["scalar"] == 3.5
        assert list(f["conv_1"].attrs["weight_names"]) == [b"conv_1_W", b"conv_1_b"]
        assert np.array_equal(f["conv_1/conv_1_W"].read(), w32)
        assert np.array_equal(f["conv_1"]["conv_1_b"].read(), np.arange(5, dtype=np.float32))
        assert np.array_equal(f["states"].read(), np.concatenate(blocks))
        fo = f["file_offsets"]
        assert len(fo) == 300
        assert tuple(fo["game_0123.sgf"].read()) == (123, 124)
        assert fo.keys() == sorted(fo.keys())


class _TinyK(H5Writer):
    LEAF_K = 2
    INTERNAL_K = 2


def test_multilevel_group_btree(tmp_path):
    p = str(tmp_path / "y.h5")
    names = ["k%03d" % i for i in range(97)]
    with _TinyK(p) as f:
        for i, n in enumerate(reversed(names)):
            f[n] = np.array([i], dtype=np.int32)
    with H5File(p) as f:
        assert f.keys() == names
        assert f["k050"].read()[0] == 96 - 50


def test_empty_chunked_dataset_has_no_chunk_records(tmp_path):
    """an empty chunked dataset is written with an UNDEF chunk-index address (as libhdf5
    does), not a fake chunk record; it reads back empty with an empty chunk index."""
    p = str(tmp_path / "empty.h5")
    with H5Writer(p) as f:
        s = f.stream_dataset("states", (3, 5, 5), np.uint8, chunk_rows=16, compression="lzf")
        s.finish()
        f.create_chunked("full", np.arange(40, dtype=np.uint8).reshape(40, 1), chunk_rows=16)
    r = H5File(p)
    d = r["states"]
    assert d.shape == (0, 3, 5, 5) and d.chunked
    assert d.chunk_index() == []
    assert d.read().shape == (0, 3, 5, 5)
    assert np.array_equal(r["full"].read().ravel(), np.arange(40))
