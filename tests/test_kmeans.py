"""k-means iterative job (BASELINE config 'k-means on 1B x 128-dim points'), CPU executors:
LocalDebug oracle vs the multi-process executor vs a numpy float64 reference."""
import numpy as np
import pytest

import dryad_amd as D
from dryad_amd import types as T
from dryad_amd.io import binary as B
from dryad_amd.models.kmeans import KMeansConfig, KMeansJob, reference
from dryad_amd.models.kmeans_cpu import gen_points

CFG = KMeansConfig(points_per_partition=1500, k=6, blobs=6, iterations=3)


def _local_debug():
    c = D.DryadLinqContext(1)
    c.LocalDebug = True
    return c


def test_points_generator_is_counter_based():
    a = gen_points(0, 50, 7, 3)
    b = gen_points(20, 30, 7, 3)
    assert a.dtype == np.float32 and a.shape == (50, 128)
    np.testing.assert_array_equal(a[20:], b)


def test_vector_type_binary_roundtrip_and_inference():
    v = tuple(float(i) / 3 for i in range(20))
    assert T.infer_type(v) == T.Vector(T.Float64, 20)
    vt = T.Vector(T.Float32, 4)
    data = B.encode_records(vt, [(1.0, 2.0, 3.0, 4.5)])
    assert len(data) == 4 + 16
    assert B.decode_records(vt, data) == [(1.0, 2.0, 3.0, 4.5)]
    # byte-compatible with a float[] field
    assert data == B.encode_records(T.ArrayT(T.Float32), [[1.0, 2.0, 3.0, 4.5]])


def test_kmeans_localdebug_matches_numpy_reference():
    r = KMeansJob(_local_debug(), CFG, partitions=2).run()
    np.testing.assert_allclose(r.centroids, reference(CFG, 2, r.iterations), rtol=0, atol=1e-6)


def test_kmeans_process_executor_matches_oracle():
    ld = KMeansJob(_local_debug(), CFG, partitions=3).run()
    ex = KMeansJob(D.DryadLinqContext(2), CFG, partitions=3).run()
    assert ex.iterations == ld.iterations
    np.testing.assert_allclose(ex.centroids, ld.centroids, rtol=0, atol=1e-6)


def test_kmeans_do_while_matches_loop():
    cfg = KMeansConfig(points_per_partition=1000, k=5, blobs=9, iterations=4)
    loop = KMeansJob(_local_debug(), cfg, partitions=2).run()
    dw = KMeansJob(_local_debug(), cfg, partitions=2).run_do_while()
    np.testing.assert_allclose(dw, loop.centroids, atol=1e-6)


def test_split_reference_is_exact_three_part():
    """The k-means split planes' twin: x == (xh + xm) + xl for every f32 magnitude, and 24-bit
    coordinates really need the third part."""
    import torch
    from dryad_amd.ops import kmeans as KM
    g = torch.Generator().manual_seed(0)
    x = torch.randn((2000, KM.DIM), generator=g) * torch.logspace(-30, 30, 2000)[:, None]
    h, m, lo = KM.split_reference(x)
    assert torch.equal((h.float() + m.float()) + lo.float(), x)
    xi = torch.randint(1 << 23, 1 << 24, (64, KM.DIM), generator=g).float()
    h, m, lo = KM.split_reference(xi)
    assert torch.equal((h.float() + m.float()) + lo.float(), xi)
    assert not torch.equal(h.float() + m.float(), xi)


def test_split_cache_follows_owner_and_version():
    import gc
    import torch
    from dryad_amd.ops import kmeans as KM
    x = torch.randn(300, KM.DIM)
    a = KM.split_points(x)
    assert KM.split_points(x[:]) is a                    # a new view of the same points hits
    x.add_(1.0)
    b = KM.split_points(x)
    assert b is not a and torch.equal(b.xh, x.bfloat16())
    n0 = len(KM._SPLITS)
    del x, a, b
    gc.collect()
    assert len(KM._SPLITS) == n0 - 1                     # the entry dies with its owner
