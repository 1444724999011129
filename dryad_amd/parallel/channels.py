"""Channel transports of the GPU executor: how a stage's port values cross between ranks.

The reference registers channel schemes (file, tcp/fifo, HDFS, managed blob; DryadVertex
channel/src/channelinterface.h and the scheme table) and the graph builder picks one per edge.
Here every cross-rank edge of an SPMD stage is one collective exchange, and the transport is
chosen per exchange from this registry: the first one that every rank can use for its values
(an all-gathered vote) moves them.

  device   device tables of one schema: RCCL all-to-all-v per column, string heaps included
           (parallel/exchange.py) -- the data plane
  object   anything else (host records left by a host fallback, structurally different tables):
           host objects through all_gather_object -- recorded, since it is a slow path

``register_transport`` adds a scheme in front of the defaults (tests, experiments).
"""
from __future__ import annotations

import torch.distributed as dist

from ..gpu.table import DeviceTable


class Transport:
    name = ""

    def usable(self, sends: list) -> bool:
        """Can this rank's values (sends[r] = values for rank r) go through this transport?"""
        raise NotImplementedError

    def move(self, runner, sends: list) -> tuple[list, str, object]:
        """All-rank exchange -> (received[r] = values from rank r, kind label, detail)."""
        raise NotImplementedError


class DeviceTransport(Transport):
    name = "device"

    def usable(self, sends):
        return all(isinstance(x, DeviceTable) for lst in sends for x in lst)

    def move(self, runner, sends):
        from . import exchange as EXC
        st = EXC.ExchangeStats()
        got = EXC.exchange(runner.world, sends, st)
        return got, "device", st.bytes_sent


class ObjectTransport(Transport):
    name = "object"

    def usable(self, sends):
        return True

    def move(self, runner, sends):
        W, me = runner.world.size, runner.world.rank
        gathered = [None] * W
        payload = [[runner._ship(x) for x in lst] for lst in sends]
        dist.all_gather_object(gathered, payload)
        # one host value per partition (aggregate partials: the reference's final-aggregate vertex
        # input) is control-plane sized; anything bigger is a data-plane object transfer
        scalar = all(isinstance(x, list) and len(x) <= 1 for lst in sends for x in lst)
        return [[runner._unship(x) for x in gathered[r][me]] for r in range(W)], \
            ("scalar" if scalar else "object"), None


_REGISTRY: list = [DeviceTransport(), ObjectTransport()]


def transports() -> list:
    return list(_REGISTRY)


def register_transport(t: Transport, first: bool = True) -> None:
    if first:
        _REGISTRY.insert(0, t)
    else:
        _REGISTRY.insert(len(_REGISTRY) - 1, t)


def unregister_transport(name: str) -> None:
    _REGISTRY[:] = [t for t in _REGISTRY if t.name != name or t.name in ("device", "object")]
