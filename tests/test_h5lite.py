"""aa_amd.h5lite against files written by the real HDF5 library
(tests/golden/make_h5.py: h5py 3.3 / HDF5 1.12): every dataset's values,
dtypes and shapes, and group listings, for the default-libver layout Keras
weight files use and for libver="latest" (object header v2, link messages,
chunked / compact / big-endian / scalar datasets)."""
from pathlib import Path

import numpy as np
import pytest

from aa_amd import h5lite

D = Path(__file__).parent / "golden" / "h5"
EXP = dict(np.load(D / "expected.npz"))


@pytest.mark.parametrize("key", sorted(EXP))
def test_dataset_values(key):
    fname, path = key.split("|", 1)
    f = h5lite.open_h5(D / f"{fname}.h5")
    got = f.read(path.replace("|", "/"))
    ref = EXP[key]
    assert got.shape == ref.shape
    assert got.dtype == ref.dtype.newbyteorder("=")
    np.testing.assert_array_equal(got, ref)


def test_groups():
    f = h5lite.open_h5(D / "keras_like.h5")
    assert sorted(f.keys()) == ["chunked", "layers", "optimizer", "vars"]
    assert sorted(f.keys("layers")) == ["batch_normalization", "conv2d", "conv2d_1", "leaky_re_lu",
                                        "mag_transform"]
    assert sorted(f.keys("layers/batch_normalization/vars")) == ["0", "1", "2", "3"]
    assert f.keys("layers/leaky_re_lu/vars") == []
    g = h5lite.open_h5(D / "many_links.h5")
    assert sorted(g.keys("g")) == [f"d{i:02d}" for i in range(40)]
    h = h5lite.open_h5(D / "latest.h5")
    assert sorted(h.keys()) == ["a", "be_f64", "compact_f32", "scalar"]


def test_rejects_non_hdf5(tmp_path):
    p = tmp_path / "x.h5"
    p.write_bytes(b"PK\x03\x04" + b"\0" * 100)
    with pytest.raises(ValueError):
        h5lite.open_h5(p)
