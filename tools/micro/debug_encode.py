"""Why does the partfile commit of a Select output not take the device encoder?"""
import sys
sys.path.insert(0, ".")
import dryad_amd as D  # noqa: E402
from dryad_amd.runtime import gpu_executor as GE  # noqa: E402
from dryad_amd.ops import codec as CD  # noqa: E402


def spy(self, s, uri, path, local):
    for p, v in local.items():
        print("part", p, type(v).__name__, v.shape.kind, v.shape.fields, {k: (str(c.dtype), tuple(c.shape)) for k, c in v.cols.items()},
              "heap", v.heap is not None, "rows", v.rows is not None, "dtype", s.dtype, flush=True)
        print("layout", CD.layout(s.dtype), flush=True)
        try:
            e = CD.encode(v, s.dtype)
            print("encode", None if e is None else tuple(e.shape), flush=True)
        except Exception as ex:  # noqa: BLE001
            print("encode raised", type(ex).__name__, ex, flush=True)
    return GE._commit_partfile_impl(self, s, uri, path, local)


GE.GpuJobRunner._commit_partfile = spy
g = D.DryadLinqContext(platform="gpu")
g.PartitionCount = 2
src = "gen://records64?count=200000&partitions=2&keys=5000&seed=3&cols=4"
g.FromStore(src).Select(lambda r: (r[0], r[1] - 7, r[2])).ToStore("partfile:///tmp/dbg_enc.pt", delete_if_exists=True).SubmitAndWait()
print("compression", g.OutputDataCompressionScheme, flush=True)
