"""Device Rabin-64 fingerprints (csrc/kernels/fingerprint.hip) against the host Rabin64 twin
(csrc/runtime/codec.cpp), and the string-pair collision check."""
import random

import pytest
import torch

pytestmark = pytest.mark.gpu


def _heap(strings):
    enc = [s.encode("utf-8") for s in strings]
    ln = torch.tensor([len(b) for b in enc], dtype=torch.int64)
    off = torch.zeros_like(ln)
    if len(enc) > 1:
        off[1:] = torch.cumsum(ln, 0)[:-1]
    blob = b"".join(enc) or b"\0"
    heap = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    return heap.cuda(), off.cuda(), ln.cuda(), enc


def test_rabin_strings_match_host():
    from dryad_amd.ops import fingerprint as F
    rng = random.Random(7)
    strings = ["", "a", "The quick brown fox", "é∂ unicode ✓"] + \
        ["".join(chr(rng.randrange(32, 127)) for _ in range(rng.randrange(0, 90))) for _ in range(3000)]
    heap, off, ln, enc = _heap(strings)
    got = F.rabin_strings(heap, off, ln).cpu().tolist()
    want = [F.rabin_host(b) for b in enc]
    assert got == want
    assert got[0] == F.signed64(F.empty())


def test_rabin_rows_match_host():
    from dryad_amd.ops import fingerprint as F
    g = torch.Generator().manual_seed(3)
    rows = torch.randint(0, 256, (5000, 100), dtype=torch.uint8, generator=g)
    got = F.rabin_rows(rows.cuda(), 3, 61).cpu().tolist()
    want = [F.rabin_host(bytes(r[3:64].tolist())) for r in rows]
    assert got == want
    full = F.rabin_rows(rows.cuda()).cpu().tolist()
    assert full[17] == F.rabin_host(bytes(rows[17].tolist()))


def test_strings_differ():
    from dryad_amd.ops import fingerprint as F
    heap, off, ln, _ = _heap(["ab", "abc", "ab", "xy", "ab"])
    trip = (heap, off, ln)
    same = torch.tensor([0, 2, 4], device="cuda")
    assert not F.strings_differ(trip, same, trip, torch.tensor([2, 4, 0], device="cuda"))
    assert F.strings_differ(trip, same, trip, torch.tensor([1, 4, 0], device="cuda"))
    assert F.strings_differ(trip, None, trip, torch.tensor([2, 1, 0, 4, 3], device="cuda"))
    assert not F.strings_differ(trip, None, trip, torch.tensor([2, 1, 0, 3, 4], device="cuda"))
