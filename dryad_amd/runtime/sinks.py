"""Output sinks of streamed stages: a stage result written piece by piece as it is produced, never
resident as a whole (SURVEY C-1: the reference's RChannelWriter writes a vertex's output as a
stream of buffers, DryadVertex/VertexHost/system/channel/include/channelinterface.h:515-723).

* ``PartfileSink``: each piece encoded on the device (fixed-width records: ops/codec.encode; records
  with strings: encode_var with a running block index) and appended through the native part writer
  (HBM -> pinned ring -> pwrite threads), to one part file or, with ``PartFileSplitBytes``, to
  SPLIT_MAX part files at once (each string file with its own block index).  ``finish()`` gives a
  ``StreamedPart`` the executor's commit renames into place.
* ``HostSink``: each piece DMA'd into leased pinned host buffers; ``finish()`` gives a
  ``HostColumns`` table the ``host://`` provider holds.

Used by the streamed aggregation (runtime/stream_agg.py) and the grace join (runtime/grace_stage.py).
"""
from __future__ import annotations

import os

import torch

from ..gpu.table import DeviceTable
from ..io.providers import parse_uri


class PartfileSink:
    def __init__(self, runner, stage, part: int, split: bool | None = None):
        from ..io import partfile as PF
        self.runner = runner
        _, path, _ = parse_uri(stage.output["uri"])
        base = PF.default_base(path)
        os.makedirs(os.path.dirname(base) or ".", exist_ok=True)
        self.tmp = f"{base}.{part:08X}---{runner.vids[stage.id][part]}_0_stream.tmp"
        self.split = int(runner.ctx.PartFileSplitBytes or 0) > 0 if split is None else split
        self.writer, self.dtype = None, None
        self.n, self.written_bytes, self.index = 0, 0, []
        self.paths = self.fbytes = self.frecs = self.findex = None
        from ..gpu.stats import BoundsAcc
        self.acc = BoundsAcc()

    @staticmethod
    def applicable(runner, stage) -> bool:
        scheme = parse_uri(stage.output["uri"])[0] if stage.is_output else None
        return scheme in ("partfile", "file") and runner.ctx.OutputDataCompressionScheme.value == 0

    def add(self, data: DeviceTable) -> bool:
        """Append one piece; False when it has no device encoding (nothing written then)."""
        from ..ops import codec as CD
        from .grace_stage import _table_dtype
        if data.n == 0 and self.writer is not None:
            return True
        if self.dtype is None:
            self.dtype = _table_dtype(data)
        enc = CD.encode(data, self.dtype) if self.dtype is not None else None
        offs = None
        if enc is None and self.dtype is not None and CD.var_layout(self.dtype) is not None:
            got = CD.encode_var(data, self.dtype, full_offsets=True)
            if got is not None:
                enc, offs = got
        if enc is None:
            return False
        B = CD.BLOCK
        if self.writer is None:
            from ..io.writer import SPLIT_MAX, PartWriter
            if self.split:
                # page-cache writes serialise per inode: SPLIT_MAX part files at once
                self.paths = [f"{self.tmp}.{j}" for j in range(SPLIT_MAX)]
                self.fbytes, self.frecs = [0] * SPLIT_MAX, [0] * SPLIT_MAX
                self.findex = [[] for _ in range(SPLIT_MAX)]
                self.writer = PartWriter(self.paths, data.device, self.runner.write_stats)
            else:
                self.writer = PartWriter(self.tmp, data.device, self.runner.write_stats)
        if self.paths is not None:
            j = min(range(len(self.fbytes)), key=self.fbytes.__getitem__)
            if offs is not None:                # block index of file j: its records n, n + B, ...
                j0 = (-self.frecs[j]) % B
                if data.n > j0:
                    self.findex[j].append(offs[j0::B] + self.fbytes[j])
            self.writer.write(enc, file=j)
            self.fbytes[j] += enc.numel()
            self.frecs[j] += data.n
        else:
            if offs is not None:                # block index of the stream: records n, n + B, ...
                j0 = (-self.n) % B
                if data.n > j0:
                    self.index.append(offs[j0::B] + self.written_bytes)
            self.writer.write(enc)
        self.acc.add(data)
        self.n += data.n
        self.written_bytes += enc.numel()
        return True

    @property
    def started(self) -> bool:
        return self.writer is not None

    def finish(self):
        """Close the writer -> (StreamedPart, bytes written)."""
        from ..io import partfile as PF
        from ..ops import codec as CD
        from .grace_stage import StreamedPart
        if self.writer is None:
            return None, 0
        if self.paths is not None:
            sizes = self.writer.close()
            keep = []
            for j, (f, b) in enumerate(zip(self.paths, sizes)):
                if b:
                    keep.append(f)
                    if self.findex[j]:
                        PF.write_index(f, self.frecs[j], b, torch.cat(self.findex[j]).cpu().numpy(), CD.BLOCK)
                else:
                    os.remove(f)
            self.writer = None
            return StreamedPart(keep or self.paths[:1], self.n, sum(sizes), self.dtype,
                                bounds=self.acc.result()), sum(sizes)
        written = self.writer.close()
        if self.index:
            PF.write_index(self.tmp, self.n, written, torch.cat(self.index).cpu().numpy(), CD.BLOCK)
        self.writer = None
        return StreamedPart(self.tmp, self.n, written, self.dtype, bounds=self.acc.result()), written

    def abort(self):
        """Stop the writer (its threads, the process-wide ring) and remove the partial files."""
        w, self.writer = self.writer, None
        if w is None:
            return
        try:
            w.abort()
        finally:
            from ..io import partfile as PF
            for f in self.paths or [self.tmp]:
                for g in (f, f + PF.INDEX_SUFFIX):
                    try:
                        os.remove(g)
                    except OSError:
                        pass


class HostSink:
    def __init__(self, runner, stage, part: int):
        self.table = None
        self.n = 0

    @staticmethod
    def applicable(runner, stage) -> bool:
        return stage.is_output and parse_uri(stage.output["uri"])[0] == "host"

    def add(self, data: DeviceTable) -> bool:
        from ..io.hosttable import HostColumns
        if data.rows is not None or data.heap is not None or data.strs:
            return False
        if self.table is None:
            self.table = HostColumns(data.shape)
        self.table.append(data)
        self.n += data.n
        return True

    @property
    def started(self) -> bool:
        return self.table is not None

    def finish(self):
        if self.table is not None and torch.cuda.is_available():
            torch.cuda.synchronize()             # every piece's DMA is done before the table is read
        return self.table, (self.table.nbytes if self.table is not None else 0)

    def abort(self):
        if self.table is not None:
            self.table.release()
        self.table = None


def for_stage(runner, stage, part: int, rest: list):
    """A sink for a streamed stage whose remaining program is only its output op, else None."""
    if [o["op"] for o in rest] != ["output"] or not stage.is_output:
        return None
    if PartfileSink.applicable(runner, stage):
        return PartfileSink(runner, stage, part)
    if HostSink.applicable(runner, stage):
        return HostSink(runner, stage, part)
    return None
