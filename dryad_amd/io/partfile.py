"""The ``partfile`` partitioned-table format (byte-compatible with the reference).

Metadata file (reference GraphManager/filesystem/DrPartitionFile.cpp:59-308, client side
LinqToDryad/DataProvider.cs:378-538):

    <partBasePath>
    <N>
    <i>,<size>[,<machine>[:<overridePath>]]      (N lines)

Partition ``i`` lives at ``<partBasePath>.%08X`` (upper-case hex of the line position).  Writers
produce ``<partBasePath>.%08X---<vertexId>_<port>_<version>.tmp`` and the job manager commits the
chosen version of each partition by rename once the whole job succeeded; other versions are deleted
(DrPartitionFile.cpp:436-600).  Parts are record streams in the DryadLinqBinary format.
"""
from __future__ import annotations

import os
import uuid
from dataclasses import dataclass, field


@dataclass
class PartEntry:
    index: int
    size: int
    machine: str | None = None
    override: str | None = None


@dataclass
class PartFileMeta:
    base: str
    parts: list = field(default_factory=list)

    @property
    def count(self) -> int:
        return len(self.parts)

    @property
    def total_size(self) -> int:
        return sum(p.size for p in self.parts)

    def part_path(self, pos: int) -> str:
        e = self.parts[pos]
        if e.override:
            return e.override
        return f"{self.base}.{pos:08X}"

    def paths(self) -> list:
        return [self.part_path(i) for i in range(self.count)]


def read_meta(meta_path: str) -> PartFileMeta:
    with open(meta_path, "r", encoding="utf-8") as f:
        lines = [ln.rstrip("\r\n") for ln in f]
    lines = [ln for ln in lines if ln.strip() != ""] if len(lines) > 2 else lines
    if len(lines) < 2:
        raise ValueError(f"the partition file {meta_path} is malformed")
    base = lines[0].strip()
    n = int(lines[1].strip())
    parts = []
    for ln in lines[2:2 + n]:
        fields = ln.split(",")
        idx, size = int(fields[0]), int(fields[1])
        machine = override = None
        if len(fields) > 2 and fields[2]:
            if ":" in fields[2]:
                machine, override = fields[2].split(":", 1)
            else:
                machine = fields[2]
        parts.append(PartEntry(idx, size, machine, override))
    if len(parts) != n:
        raise ValueError(f"the partition file {meta_path} is malformed: expected {n} parts, found {len(parts)}")
    if not os.path.isabs(base):
        base = os.path.join(os.path.dirname(os.path.abspath(meta_path)), base)
    return PartFileMeta(base, parts)


def write_meta(meta_path: str, meta: PartFileMeta):
    tmp = meta_path + ".tmp-" + uuid.uuid4().hex[:8]
    with open(tmp, "w", encoding="utf-8", newline="\n") as f:
        f.write(meta.base + "\n")
        f.write(f"{meta.count}\n")
        for i, p in enumerate(meta.parts):
            extra = ""
            if p.machine:
                extra = "," + p.machine + (":" + p.override if p.override else "")
            f.write(f"{i},{p.size}{extra}\n")
    os.replace(tmp, meta_path)


def default_base(meta_path: str) -> str:
    d = os.path.dirname(os.path.abspath(meta_path))
    name = os.path.basename(meta_path)
    return os.path.join(d, name + ".parts", "Part")


def tmp_part_path(base: str, pos: int, vertex_id: int, port: int, version: int) -> str:
    return f"{base}.{pos:08X}---{vertex_id}_{port}_{version}.tmp"


def commit_parts(meta_path: str, base: str, chosen: list[str], machine: str | None = None) -> PartFileMeta:
    """Rename the chosen temporary part files to their final names and write the metadata."""
    os.makedirs(os.path.dirname(base), exist_ok=True)
    parts = []
    for pos, src in enumerate(chosen):
        dst = f"{base}.{pos:08X}"
        if src != dst:
            os.replace(src, dst)
            if os.path.exists(src + INDEX_SUFFIX):
                os.replace(src + INDEX_SUFFIX, dst + INDEX_SUFFIX)
            elif os.path.exists(dst + INDEX_SUFFIX):
                os.remove(dst + INDEX_SUFFIX)      # a stale index of an earlier version
        parts.append(PartEntry(pos, os.path.getsize(dst), machine))
    meta = PartFileMeta(base, parts)
    write_meta(meta_path, meta)
    return meta


def cleanup_tmp(base: str):
    """Delete every uncommitted ``.tmp`` version of ``base`` (failed / duplicate vertices)."""
    d = os.path.dirname(base)
    if not os.path.isdir(d):
        return
    prefix = os.path.basename(base) + "."
    for fn in os.listdir(d):
        if fn.startswith(prefix) and fn.endswith(".tmp") and "---" in fn:
            try:
                os.remove(os.path.join(d, fn))
            except OSError:
                pass


def exists(meta_path: str) -> bool:
    return os.path.exists(meta_path)


# Replaced tables recycle their part files.  A table replaced by ToStore(delete_if_exists=True)
# usually has a successor of about the same size written into the same directory; its parts are
# renamed into ``<parts dir>/.recycle/`` instead of being unlinked, and the writer of a new part
# claims one (atomic rename, so ranks sharing the directory never claim the same file) and
# overwrites it in place (io/writer.write_device_pieces(reuse=True)).  Unlinking a page-cached part
# frees its pages, and writing a fresh one allocates them again: 15 GB written into fresh files
# while the previous 15 GB are unlinked runs at a fraction of the writer's rate
# (tools/micro/writeback_probe2.py).  Files nobody claims within RECYCLE_TTL seconds are unlinked
# by a daemon thread (and by the next delete's sweep, after a restart).
RECYCLE_DIR = ".recycle"
RECYCLE_TTL = 60.0
_MINE: set = set()            # recycled files this process created (unlinked at exit if unclaimed)
_ATEXIT = False


def _remember(path: str) -> None:
    """Track a recycled file; the first one registers the exit hook that unlinks what nobody
    claimed (a short script, or a failed write whose commit never dropped them, exits before the
    daemon thread's TTL)."""
    global _ATEXIT
    _MINE.add(path)
    if not _ATEXIT:
        import atexit
        atexit.register(_drop_mine)
        _ATEXIT = True


def _drop_mine() -> None:
    for q in list(_MINE):
        try:
            os.remove(q)                 # claimed ones were renamed away: nothing to remove
        except OSError:
            pass
    _MINE.clear()


def _recycle_dir(path: str) -> str:
    return os.path.join(os.path.dirname(path), RECYCLE_DIR)


def _sweep(d: str, older_than: float):
    import time
    now = time.time()
    try:
        names = os.listdir(d)
    except OSError:
        return
    for fn in names:
        try:
            stamp = int(fn.split("-")[1]) / 1e3
        except (IndexError, ValueError):
            continue
        if now - stamp >= older_than:
            try:
                os.remove(os.path.join(d, fn))
            except OSError:
                pass


def claim_recycled(paths: list) -> int:
    """Rename recycled part files (the largest first) onto ``paths`` (new part files of one
    directory that do not exist yet); returns how many were claimed.  The writer then overwrites
    them in place and cuts them to size."""
    if not paths:
        return 0
    d = _recycle_dir(paths[0])
    try:
        cands = sorted(((os.path.getsize(os.path.join(d, fn)), fn) for fn in os.listdir(d)
                        if fn.startswith("r-")), reverse=True)
    except OSError:
        return 0
    got = 0
    it = iter(cands)
    for p in paths:
        if os.path.exists(p):
            continue
        for _, fn in it:
            try:
                os.rename(os.path.join(d, fn), p)
            except OSError:          # claimed by another rank meanwhile
                continue
            got += 1
            break
        else:
            break
    return got


def drop_recycled(base: str):
    """Unlink (on a daemon thread) the recycled files of ``base``'s parts directory that the table
    just written there did not claim: they would only hold disk space until their TTL."""
    d = _recycle_dir(base)
    if not os.path.isdir(d):
        return
    import threading
    threading.Thread(target=_sweep, args=(d, 0.0), daemon=True, name="dryad-recycle-drop").start()


def delete(meta_path: str, background: bool = False, recycle: bool = True):
    """Delete the table: every partition then the metadata (CheckExistence(deleteIfExists)).
    ``background``: the files are renamed out of the way at once (the table is gone and its
    names are free for a new one); with ``recycle`` the part files go to the recycle directory of
    their parts directory (see RECYCLE_DIR), everything else is unlinked by a daemon thread:
    unlinking tens of GB of page-cached parts takes seconds the job does not have to wait for."""
    if not os.path.exists(meta_path):
        return
    if background:
        import threading
        import time
        tag = ".deleting-" + uuid.uuid4().hex[:8]
        stamp = int(time.time() * 1e3)
        moved, recycled = [], []
        rdir = None
        try:
            meta = read_meta(meta_path)
            for i, p in enumerate(meta.paths()):
                if recycle and os.path.exists(p):
                    rdir = _recycle_dir(p)
                    os.makedirs(rdir, exist_ok=True)
                    q = os.path.join(rdir, f"r-{stamp}-{uuid.uuid4().hex[:8]}-{i}")
                    os.replace(p, q)
                    recycled.append(q)
                    _remember(q)
                elif os.path.exists(p):
                    os.replace(p, p + tag)
                    moved.append(p + tag)
                if os.path.exists(p + INDEX_SUFFIX):
                    os.replace(p + INDEX_SUFFIX, p + INDEX_SUFFIX + tag)
                    moved.append(p + INDEX_SUFFIX + tag)
        except Exception:
            pass
        os.replace(meta_path, meta_path + tag)
        moved.append(meta_path + tag)

        def unlink_all():
            for q in moved:
                try:
                    os.remove(q)
                except OSError:
                    pass
            if rdir is not None:
                _sweep(rdir, 10 * RECYCLE_TTL)      # leftovers of an earlier process
                time.sleep(RECYCLE_TTL)
                for q in recycled:                  # not claimed by a successor
                    try:
                        os.remove(q)
                    except OSError:
                        pass
        threading.Thread(target=unlink_all, daemon=True, name="dryad-partfile-delete").start()
        return
    try:
        meta = read_meta(meta_path)
        for p in meta.paths():
            if os.path.exists(p):
                os.remove(p)
            if os.path.exists(p + INDEX_SUFFIX):
                os.remove(p + INDEX_SUFFIX)
    except Exception:
        pass
    os.remove(meta_path)


# ------------------------------------------------------------------------------------------------
# Record block index sidecar (``<part>.idx``): the byte offset of every B-th record of a part of
# variable-length records, so the device decoder (ops/codec.decode_var) parses the blocks in
# parallel without a sequential scan of the part.  Written next to the part by the writers that
# know the record boundaries (io/binary.write_records, the device encoder); absent for parts
# written elsewhere (the reader then scans the part on the host: codec.cpp scan_record_blocks).
# Layout (little endian): b"DRIX", u32 version = 1, u32 B, u64 records, u64 part bytes,
# u64 offsets[ceil(records / B)].
INDEX_SUFFIX = ".idx"
_INDEX_MAGIC = b"DRIX"


def write_index(part_path: str, n: int, nbytes: int, offsets, block: int) -> None:
    import struct
    import numpy as np
    offs = np.ascontiguousarray(np.asarray(offsets, dtype="<u8"))
    with open(part_path + INDEX_SUFFIX, "wb") as f:
        f.write(_INDEX_MAGIC + struct.pack("<IIQQ", 1, int(block), int(n), int(nbytes)))
        f.write(offs.tobytes())


def read_index(part_path: str):
    """(records, part bytes, B, int64 offsets) of a part's index, or None when absent / stale."""
    import struct
    import numpy as np
    p = part_path + INDEX_SUFFIX
    if not os.path.exists(p):
        return None
    with open(p, "rb") as f:
        head = f.read(28)
        if len(head) != 28 or head[:4] != _INDEX_MAGIC:
            return None
        ver, block, n, nbytes = struct.unpack("<IIQQ", head[4:])
        if ver != 1 or block == 0 or nbytes != os.path.getsize(part_path):
            return None
        offs = np.frombuffer(f.read(), dtype="<u8").astype(np.int64)
    if offs.shape[0] != (n + block - 1) // block:
        return None
    # offsets a block-parallel decoder may trust: from 0, never decreasing, inside the part
    if offs.shape[0] and (offs[0] != 0 or (offs[1:] < offs[:-1]).any() or offs[-1] > nbytes or offs[-1] < 0):
        return None
    return int(n), int(nbytes), int(block), offs
