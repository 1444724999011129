"""Recycled part files of a replaced table that no successor claimed are unlinked when the
process exits (a short script used to leave tens of GB in .recycle/)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _recycled(tmp_path):
    out = []
    for root, _, files in os.walk(tmp_path):
        if os.path.basename(root) == ".recycle":
            out += files
    return out


def test_unclaimed_recycled_parts_go_at_exit(tmp_path):
    code = (f"import sys; sys.path.insert(0, {ROOT!r})\n"
            "from dryad_amd.io import partfile as PF\n"
            "from dryad_amd.io.providers import provider_for\n"
            f"uri = 'partfile://{tmp_path}/t.pt'\n"
            "provider_for(uri).write_table(uri, [b'x' * 1000, b'y' * 1000], None)\n"
            f"PF.delete('{tmp_path}/t.pt', background=True)\n"
            "print(len(PF._MINE))\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr[-2000:]
    assert int(out.stdout.strip().splitlines()[-1]) == 2, out.stdout     # both parts were recycled ...
    assert _recycled(tmp_path) == []                                      # ... and unlinked at exit
