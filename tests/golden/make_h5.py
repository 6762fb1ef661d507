"""Write HDF5 fixtures with the real HDF5 library, to pin aa_amd/h5lite.py.

Run with an interpreter that has h5py (this image's /opt/conda/bin/python3.9
does; the build's own Python does not):

    cd /tmp && /opt/conda/bin/python3.9 /root/repo/tests/golden/make_h5.py

Writes tests/golden/h5/*.h5 plus expected.npz (every dataset's values):
* keras_like.h5  -- the layout Keras 3 gives model.weights.h5
  (layers/<snake_case class name>[_k]/vars/<i>, top-level vars/), default
  libver (superblock 0, object header v1, symbol-table groups), contiguous
  plus one chunked dataset (B-tree v1 chunk index)
* latest.h5      -- libver="latest" (superblock 3, object header v2, compact
  link messages, layout message v4), compact / contiguous / big-endian /
  scalar datasets (v4 chunk indexes are not read)
* many_links.h5  -- a symbol-table group with 40 members (B-tree with
  several leaves)
"""
import os
import sys

import h5py
import numpy as np

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "h5")
os.makedirs(OUT, exist_ok=True)
rng = np.random.default_rng(7)
expected = {}


def ds(g, name, arr, key, **kw):
    g.create_dataset(name, data=arr, **kw)
    expected[key] = np.asarray(arr)


with h5py.File(os.path.join(OUT, "keras_like.h5"), "w") as f:
    f.create_group("vars")
    L = f.create_group("layers")
    for lname, shapes in (("conv2d", [(3, 3, 1, 4), (4,)]), ("batch_normalization", [(4,)] * 4),
                          ("conv2d_1", [(1, 1, 4, 3)]), ("mag_transform", [(1,)])):
        v = L.create_group(lname).create_group("vars")
        for i, sh in enumerate(shapes):
            ds(v, str(i), rng.standard_normal(sh).astype(np.float32), f"keras_like/layers/{lname}/vars/{i}")
    L.create_group("leaky_re_lu").create_group("vars")
    f.create_group("optimizer").create_group("vars")
    ds(f, "chunked", rng.standard_normal((37, 11)).astype(np.float32), "keras_like/chunked", chunks=(8, 4))

with h5py.File(os.path.join(OUT, "latest.h5"), "w", libver="latest") as f:
    g = f.create_group("a/b")
    ds(g, "contig_i32", np.arange(-5, 7, dtype=np.int32), "latest/a/b/contig_i32")
    ds(f, "be_f64", np.linspace(-1, 1, 9).astype(">f8"), "latest/be_f64")
    ds(f, "scalar", np.float32(3.5), "latest/scalar")
    dcpl = h5py.h5p.create(h5py.h5p.DATASET_CREATE)
    dcpl.set_layout(h5py.h5d.COMPACT)
    arr = np.arange(6, dtype=np.float32).reshape(2, 3) / 7
    space = h5py.h5s.create_simple(arr.shape)
    dsid = h5py.h5d.create(f.id, b"compact_f32", h5py.h5t.NATIVE_FLOAT, space, dcpl=dcpl)
    dsid.write(h5py.h5s.ALL, h5py.h5s.ALL, arr)
    expected["latest/compact_f32"] = arr

with h5py.File(os.path.join(OUT, "many_links.h5"), "w") as f:
    g = f.create_group("g")
    for i in range(40):
        ds(g, f"d{i:02d}", np.full((i % 5 + 1,), i, dtype=np.float64), f"many_links/g/d{i:02d}")

np.savez(os.path.join(OUT, "expected.npz"), **{k.replace("/", "|"): v for k, v in expected.items()})
print("wrote", sorted(os.listdir(OUT)), file=sys.stderr)
