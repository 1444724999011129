"""DeviceTable packing for the all-to-all (gpu/table.py) on CPU tensors: pack / unpack_like round
trips, including the zero-row receive a rank gets when no key range of a shuffle lands on it."""
import torch

from dryad_amd.gpu.table import DeviceTable, Shape


def test_pack_unpack_round_trip_and_empty_receive():
    t = DeviceTable.from_columns({"a": torch.arange(5), "b": torch.arange(5).double(),
                                  "v": torch.arange(15, dtype=torch.float32).reshape(5, 3)},
                                 Shape("tuple", ["a", "b", "v"]))
    p = t.pack()
    assert p.shape == (5, 8 + 8 + 12)
    u = t.unpack_like(p.reshape(-1), 5)
    for k in t.cols:
        assert torch.equal(u.cols[k], t.cols[k])
    e = t.unpack_like(torch.empty(0, dtype=torch.uint8), 0)
    assert e.n == 0 and e.cols["v"].shape == (0, 3) and e.cols["b"].dtype == torch.float64
    rows = DeviceTable(3, Shape("rows", key_off=0, key_len=4), rows=torch.zeros((3, 16), dtype=torch.uint8))
    assert rows.unpack_like(torch.empty(0, dtype=torch.uint8), 0).rows.shape == (0, 16)


def test_pack_of_empty_expanded_column():
    t = DeviceTable.from_columns({"a": torch.zeros(1, dtype=torch.int32).expand(0), "b": torch.empty(0)},
                                 Shape("tuple", ["a", "b"]))
    assert t.pack().shape == (0, 8)


def test_unpack_single_row():
    t = DeviceTable.from_columns({"i": torch.tensor([7], dtype=torch.int32), "d": torch.tensor([2.5]),
                                  "j": torch.tensor([-3], dtype=torch.int64), "e": torch.tensor([1.5])},
                                 Shape("tuple", ["i", "d", "j", "e"]))
    u = t.unpack_like(t.pack().reshape(-1), 1)
    assert [u.cols[k].tolist() for k in "idje"] == [[7], [2.5], [-3], [1.5]]
