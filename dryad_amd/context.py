"""``DryadLinqContext``: job configuration and the factory for query inputs.

Reference: LinqToDryad/DryadLinqContext.cs:566-1310.  Constructors map to the MI355X node:

  * ``DryadLinqContext(num_processes)``        LOCAL platform: the job manager plus
    ``num_processes`` CPU worker processes on this host (LocalJobSubmission analog, used for the
    WordCount plumbing config and CI without a GPU)
  * ``DryadLinqContext(platform="gpu")``       GPU platform: SPMD over the ranks of the current
    ``torchrun`` world, one MI355X per rank, RCCL over xGMI for shuffles
  * ``DryadLinqContext(cluster=LocalGpuNode(n))`` explicit cluster descriptor

Configuration properties keep the reference names (``JobFriendlyName``, ``EnableSpeculativeDuplication``,
``LocalDebug``, ...) and are frozen once the context has run a job (test ContextConfigIsReadOnly).
"""
from __future__ import annotations

import enum
import itertools
import os
import threading

from . import types as T
from .errors import DryadLinqException, ErrorCode
from .jobinfo import DryadLinqJobInfo, JobHandle, JobStatus
from .query import Query, QNode


class PlatformKind(enum.Enum):
    LOCAL = "LOCAL"          # CPU worker processes on this host
    GPU = "GPU"              # MI355X ranks of a torchrun world
    LOCAL_DEBUG = "LOCAL_DEBUG"


class ExecutorKind(enum.Enum):
    DRYAD = "DRYAD"
    LOCAL_DEBUG = "LOCAL_DEBUG"


class CompressionScheme(enum.Enum):
    NONE = 0
    GZIP = 1
    None_ = 0


class QueryLoggingLevel(enum.IntEnum):
    """Reference QueryTraceLevel.cs:30-37 / Constants.cs:72-112 (bit masks)."""
    Off = 0
    Critical = 1
    Error = 3
    Warning = 7
    Information = 15
    Verbose = 31


class DryadLinqCluster:
    """Cluster descriptor interface (reference DryadLinqContext.cs:76-106)."""
    platform = PlatformKind.LOCAL

    def make_context_defaults(self) -> dict:
        return {}


class LocalCpuCluster(DryadLinqCluster):
    platform = PlatformKind.LOCAL

    def __init__(self, num_processes: int = 2):
        self.num_processes = int(num_processes)


class LocalGpuNode(DryadLinqCluster):
    """One MI355X node: ``n_gpus`` ranks (defaults to the torchrun WORLD_SIZE)."""
    platform = PlatformKind.GPU

    def __init__(self, n_gpus: int | None = None):
        self.n_gpus = n_gpus


_ctx_ids = itertools.count(1)

_DEFAULTS = dict(
    IntermediateDataCompressionScheme=CompressionScheme.NONE,
    OutputDataCompressionScheme=CompressionScheme.NONE,
    CompileForVertexDebugging=False,
    JobFriendlyName="DryadLINQ job",
    JobMinNodes=None,
    JobMaxNodes=None,
    ThreadsPerWorker=None,
    JobRuntimeLimit=None,
    EnableSpeculativeDuplication=True,
    OutlierThresholdSeconds=None,      # a vertex running past it gets a duplicate (None: the stage's
    #                                    non-parametric estimate, >= 10 s; DrStageStatistics.cpp:93-111)
    LocalDebug=False,
    DebugBreak=False,
    RuntimeLoggingLevel=QueryLoggingLevel.Error,
    SelectOrderPreserving=False,
    ForceGC=False,
    PartitionCount=None,               # default partition count for shuffles (StaticConfig 8)
    MaxVertexFailures=6,               # DrGraphParameters: m_maxActiveFailureCount
    DynamicOptLevel=0x1,               # broadcast only (DryadLinqGlobals.cs:43-52)
    AggregationTreeMaxInputs=150,      # aggregation tree: max inputs per vertex (DryadLinqApplication.cs:173-175)
    AggregationTreeGroup=32,           # ... and partials folded per interior vertex
    AggregateThreshold=1 << 30,        # dynamic aggregation: bytes per combine vertex (the GM's
                                       # at/aggregatethreshold, DryadLinqApplication.cs:143-175; "512MB" ok)
    HeadNode="localhost",
    DryadHomeDirectory=None,
    PartitionUncPath=None,
    Queue=None,
    NodeGroup=None,
    ContainerMbMemory=None,
    ApplicationMasterMbMemory=None,
    GraphManagerNode=None,
    FaultInjection=None,          # [{stage, partition, version, kind}] (SURVEY §5.3 FaultInjector)
    HbmBudgetBytes=None,          # HBM an out-of-core operator may use per GPU (None: 80% of free HBM)
    ExternalSort=None,            # out-of-core OrderBy to host:// (None: when the data exceeds the budget)
    AllowHostFallback=False,      # GPU executor: an op whose lambdas do not trace may run on host
    HostFallbackMaxBytes=256 << 20,  # ... records only up to this many partition bytes unless allowed
    RerunInputsMaxBytes=1 << 30,  # inputs a failed GPU vertex's restart record may persist
    ExternalSortToDisk=None,      # its partfile:// output written through a memory-mapped part file
    #                               (None: when the output exceeds half of the available host memory)
    StreamStages=None,            # read -> record-wise ops -> partfile stages chunk-streamed (runtime/
    #                               streaming.py; None: when a source partition exceeds StreamChunkBytes)
    StreamChunkBytes=4 << 30,     # ... and their chunk size
    StreamAggregate=None,         # read -> GroupBy / Distinct stages folded chunk by chunk in bounded HBM
    #                               (runtime/stream_agg.py; None: when a partition exceeds HbmBudgetBytes)
    StreamDenseState=True,        # ... a streamed GroupBy of one integer key keeps its running state
    #                               directly addressed by key while the keys' range fits the budget
    StreamShuffle=None,           # multi-partition GroupBy / Distinct: partial side, exchange and final
    #                               side as pipelined rounds with bounded channels (runtime/
    #                               stream_shuffle.py; None: when a source partition exceeds the budget)
    GraceJoin=None,               # a Join as the partitioned grace join stage (runtime/grace_stage.py;
    #                               None: when its inputs would crowd the HBM budget; False: never)
    GraceJoinStringBytes=64,      # ... inline bytes per string field in its packed bucket rows, at least
    #                               (longer strings widen the rows; past 512-byte rows the compiled join runs)
    LineAlignedSortInput=True,   # GPU executor: a table of 100-byte rows that only an OrderBy reads is
    #                               stored at a 128-byte pitch (one HBM line per record gather)
    GenFusedShuffle=False,        # multi-rank OrderBy over gen://terasort: generate the records straight
    #                               into the exchange's send rows (no input table; a benchmark variant)
    GroupByAggregation="auto",    # single-integer-key GroupBy: "auto" (radix aggregation for keys spanning
    #                               >= 2^32 values), "radix" or "sort" (ops/tuning.py)
    ShuffleSlack=0.01,            # receive-buffer headroom of a range-partitioned exchange
    ExchangeOneRank=False,        # plan a one-partition OrderBy as the sampled range shuffle, so a one-rank
    #                               RCCL communicator (World.force_collectives) runs the multi-rank program
    PersistStageOutputs=None,     # GPU executor: copy completed stage outputs to a checkpoint store so a
    #                               relaunched gang resumes there (None: under a relaunching launcher;
    #                               a directory or True: always; False: never; runtime/checkpoint.py)
    CheckpointBudgetBytes=None,   # ... bytes the persisted outputs may take (None: 90% of the checkpoint
    #                               file system's free space); a stage past it is not persisted
    PartFileSplitBytes=0,         # GPU executor: a fixed-width partfile:// output partition of at least
    #                               this many bytes is written as several part files at once (0: one
    #                               part file per partition, as the reference; io/writer.split_count)
)

_READONLY_AFTER_USE = set(_DEFAULTS) - {"LocalDebug"}


class DryadLinqContext:
    def __init__(self, num_processes: int | None = None, storage_set_scheme: str | None = None, *,
                 platform: str | PlatformKind | None = None, cluster: DryadLinqCluster | None = None,
                 temp_dir: str | None = None):
        object.__setattr__(self, "_props", dict(_DEFAULTS))
        object.__setattr__(self, "_frozen", False)
        object.__setattr__(self, "_id", next(_ctx_ids))
        self._props["JobEnvironmentVariables"] = {}
        self._props["ResourcesToAdd"] = []
        self._props["ResourcesToRemove"] = []
        if isinstance(platform, str):
            platform = PlatformKind(platform.upper())
        if cluster is not None:
            platform = cluster.platform
            if isinstance(cluster, LocalCpuCluster):
                num_processes = cluster.num_processes
        if platform is None:
            platform = PlatformKind.LOCAL
        self._props["PlatformKind"] = platform
        self._props["ExecutorKind"] = ExecutorKind.DRYAD
        self._props["NumProcesses"] = int(num_processes) if num_processes else 2
        self._props["StorageScheme"] = storage_set_scheme or ("hbm" if platform == PlatformKind.GPU else "partfile")
        self._props["TempDir"] = temp_dir
        object.__setattr__(self, "_cluster", cluster)
        object.__setattr__(self, "_lock", threading.RLock())
        object.__setattr__(self, "_executor", None)
        object.__setattr__(self, "_jobs", {})
        object.__setattr__(self, "_job_seq", itertools.count(1))

    # ------------------------------------------------------------------ properties
    def __getattr__(self, name):
        props = object.__getattribute__(self, "_props")
        if name in props:
            return props[name]
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name in self._props or name in _DEFAULTS:
            if self._frozen and name in _READONLY_AFTER_USE:
                raise DryadLinqException(ErrorCode.Unspecified, f"DryadLinqContext.{name} cannot be changed after the context was used")
            self._props[name] = value
        else:
            object.__setattr__(self, name, value)

    @property
    def num_partitions(self) -> int:
        if self.PartitionCount:
            return int(self.PartitionCount)
        if self.PlatformKind == PlatformKind.GPU:
            from .parallel.comm import get_world
            return max(1, get_world().size)
        return max(1, int(self.NumProcesses))

    def _compatible(self, other) -> bool:
        return isinstance(other, DryadLinqContext) and other._props["PlatformKind"] == self._props["PlatformKind"]

    def __eq__(self, other):
        return self is other

    def __hash__(self):
        return self._id

    def Dispose(self):
        """Release the executor; any later use of the context raises ContextDisposed
        (reference DryadLinqContext.Dispose / ThrowIfDisposed, DryadLinqContext.cs:1262-1275)."""
        object.__setattr__(self, "_disposed", True)
        if self._executor is not None:
            self._executor.close()
            object.__setattr__(self, "_executor", None)

    def _throw_if_disposed(self):
        if getattr(self, "_disposed", False):
            raise DryadLinqException(ErrorCode.ContextDisposed, "the DryadLinqContext has been disposed")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.Dispose()

    def ClientVersion(self):
        self._throw_if_disposed()
        from . import __version__
        return __version__

    def ServerVersion(self):
        """Version of the job-side runtime (the native job graph library when built)."""
        self._throw_if_disposed()
        from . import __version__
        return __version__

    # ------------------------------------------------------------------ inputs
    def FromEnumerable(self, data, dtype=None) -> Query:
        self._throw_if_disposed()
        data = list(data)
        if dtype is None:
            dtype = T.infer_common_type(data[:1000]) if data else T.Int32
        return Query(self, QNode("FromEnumerable", (), dict(data=data), dtype))

    def FromStore(self, uri: str, dtype=None, deserializer=None) -> Query:
        from .io.providers import provider_for
        self._throw_if_disposed()
        p = provider_for(str(uri))
        if not p.exists(str(uri)):
            raise DryadLinqException(ErrorCode.FailedToGetStreamProps, f"dataset {uri} does not exist")
        if dtype is None:
            dtype = T.LineRecordT if str(uri).startswith("partfile") and deserializer is None else None
            sch = p.schema(str(uri)) if hasattr(p, "schema") else None
            if sch is not None and sch.get("dtype") is not None:
                dtype = sch["dtype"]
        else:
            dtype = T.from_annotation(dtype)
        return Query(self, QNode("FromStore", (), dict(uri=str(uri), deserializer=deserializer), dtype))

    def MakeTemporaryStreamUri(self) -> str:
        from .io.providers import provider_for, unique_name
        scheme = self.StorageScheme
        return provider_for(scheme + "://x").temp_uri(unique_name("DryadLinqTemp"))

    # ------------------------------------------------------------------ execution
    def _freeze(self):
        object.__setattr__(self, "_frozen", True)

    def _get_executor(self):
        if self._executor is None:
            with self._lock:
                if self._executor is None:
                    from .runtime.executor import make_executor
                    object.__setattr__(self, "_executor", make_executor(self))
        return self._executor

    def _local_debug(self) -> bool:
        return bool(self.LocalDebug) or self.PlatformKind == PlatformKind.LOCAL_DEBUG

    def _write_local_store(self, node: QNode, data):
        from .io.providers import provider_for
        uri = node.args["uri"]
        p = provider_for(uri)
        if p.exists(uri) and not node.args.get("delete_if_exists") and not node.args.get("_temp"):
            raise DryadLinqException(ErrorCode.StreamAlreadyExists, f"can't output to existing table {uri}")
        dtype = node.dtype or (T.infer_common_type(data[:1000]) if data else T.Int32)
        node.dtype = dtype
        p.write_table(uri, [data], dtype)

    def _enumerate(self, q: Query) -> list:
        self._throw_if_disposed()
        self._freeze()
        if self._local_debug():
            from .localdebug import LocalEvaluator
            return LocalEvaluator(self).eval(q.node)
        return self._get_executor().enumerate(q)

    def _execute_scalar(self, q: Query):
        self._throw_if_disposed()
        self._freeze()
        if self._local_debug():
            from .localdebug import LocalEvaluator
            return LocalEvaluator(self).eval(q.node)[0]
        res = self._get_executor().enumerate(q)
        if len(res) != 1:
            raise DryadLinqException(ErrorCode.SingleMoreThanOneElement, f"scalar query produced {len(res)} records")
        return res[0]

    def _new_handle(self) -> JobHandle:
        return JobHandle(f"{self._id}.{next(self._job_seq)}")

    def Submit(self, *queries) -> DryadLinqJobInfo:
        """Submit one or several ``ToStore`` queries as ONE job (reference Submit(params IQueryable[]))."""
        qs = []
        for q in queries:
            qs.extend(q if isinstance(q, (list, tuple)) else [q])
        self._throw_if_disposed()
        for q in qs:
            if not isinstance(q, Query):
                raise DryadLinqException(ErrorCode.MustStartFromContext,
                                         "only DryadLINQ queries created from a DryadLinqContext can be submitted")
            if q._ctx is not self:
                raise DryadLinqException(ErrorCode.MustStartFromContext,
                                         "the queries submitted together must be created using the same DryadLinqContext")
        self._freeze()
        outs = []
        for q in qs:
            if q.node.op != "ToStore":
                q = q.ToStore(self.MakeTemporaryStreamUri())
                q.node.args["_temp"] = True
            outs.append(q)
        # repeat submission of an executed query returns the existing job
        key = tuple(sorted(q.node.id for q in outs))
        prev = self._jobs.get(key)
        if prev is not None:
            return prev
        h = self._new_handle()
        info = DryadLinqJobInfo([h])
        self._jobs[key] = info
        if self._local_debug():
            from .localdebug import LocalEvaluator
            try:
                ev = LocalEvaluator(self)
                for q in outs:
                    ev.eval(q.node)
                h.finish(True)
            except BaseException as e:  # noqa: BLE001
                h.finish(False, e)
            return info
        self._get_executor().submit(outs, h)
        return info

    def SubmitAndWait(self, *queries) -> DryadLinqJobInfo:
        info = self.Submit(*queries)
        info.Wait()
        return info

    def _do_while(self, source: Query, body, cond, checkpoint: str | None = None) -> Query:
        """Client loop of DoWhile.  Every iteration is materialised (reference
        DryadLinqQueryable.cs:1297-1305); with ``checkpoint`` (a partfile/text/hbm uri prefix) the
        iterations are persistent tables ``<checkpoint>.iter<k>`` plus a state file, and a rerun
        of the same loop resumes after the last completed iteration."""
        import json as _json
        before = source
        k = 0
        state_path = None
        if checkpoint is not None:
            from .io.providers import parse_uri
            scheme, path, _ = parse_uri(checkpoint)
            if scheme in ("partfile", "file", "text"):
                state_path = path + ".dowhile.json"
            else:
                state_path = os.path.join(os.environ.get("TMPDIR", "/tmp"),
                                          "dryad-dowhile-" + checkpoint.replace("/", "_").replace(":", "_") + ".json")
            if os.path.exists(state_path):
                with open(state_path) as f:
                    st = _json.load(f)
                before = self.FromStore(st["table"])
                k = st["iteration"]
                if st.get("done"):
                    return before
        while True:
            after = body(before)
            if not self._local_debug():
                if checkpoint is not None:
                    tmp = f"{checkpoint}.iter{k + 1}"
                    st = after.ToStore(tmp, delete_if_exists=True)
                else:
                    tmp = self.MakeTemporaryStreamUri()
                    st = after.ToStore(tmp)
                    st.node.args["_temp"] = True
                self.SubmitAndWait(st)
                after = Query(self, QNode("Table", (), dict(uri=tmp), st.node.dtype))
            else:
                after = self.FromEnumerable(list(after), dtype=after.dtype)
            more = cond(before, after)
            val = more.Single() if isinstance(more, Query) else bool(more)
            k += 1
            if state_path is not None and not self._local_debug():
                prev = before.node.args.get("uri") if before.node.op in ("Table", "FromStore") else None
                tmp_state = state_path + ".tmp"
                with open(tmp_state, "w") as f:
                    _json.dump(dict(iteration=k, table=after.node.args["uri"], done=not val), f)
                os.replace(tmp_state, state_path)          # commit the iteration
                if prev and prev.startswith(f"{checkpoint}.iter"):
                    from .io.providers import provider_for
                    try:
                        provider_for(prev).delete(prev)
                    except Exception:  # noqa: BLE001
                        pass
            if not val:
                return after
            before = after

    def Explain(self, q: Query) -> str:
        from .compiler.planner import compile_queries
        plan = compile_queries(self, [q])
        return plan.explain()

    # python-style aliases
    from_enumerable = FromEnumerable
    from_store = FromStore
    submit = Submit
    submit_and_wait = SubmitAndWait
