"""Physical query plan: stages (vertex sets), their inputs/connections and vertex programs.

Mirrors the reference XML query plan (LinqToDryad/DryadLinqQueryGen.cs:837-971,
DryadLinqQueryNode.cs:728-827): every plan vertex has UniqueId, Type, Name, Explain, Partitions,
ChannelType, ConnectionOperator, DynamicManager, Entry and Children.  Here a ``Stage`` is one
vertex set; ``StageInput.kind`` is the connection operator:

  * ``pointwise``  vertex p reads partition p of the source (same partition count)
  * ``cross``      CrossProduct: vertex p reads output port p of *every* source vertex (shuffle)
  * ``merge``      N -> 1: the single vertex reads port ``port`` of every source vertex in order
  * ``broadcast``  every vertex reads port ``port`` of every source vertex (Tee + CrossProduct)
  * ``offset``     vertex p reads source partition p - offset if it exists (Concat)

A vertex program is a list of op dicts executed in sequence by the vertex runtime; the first op
receives all stage inputs, later ops the previous op's single output stream.  The last op may emit
several output ports (partitioners, Fork).
"""
from __future__ import annotations

import json
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

from .datasetinfo import DataSetInfo

CHANNEL_TYPES = ("DiskFile", "HBM", "MemoryFIFO")


@dataclass
class StageInput:
    src: int
    kind: str = "pointwise"
    port: int = 0
    offset: int = 0
    merge_sort: dict | None = None      # k-way merge of sorted source ports: {key, comparer, descending}
    group: int = 0                      # kind "group": partition j reads source partitions [j*g, (j+1)*g)
    dynamic: bool = False               # kind "group": regroup by the sources' output sizes at run time
                                        # (runtime/aggmanager.py; the static groups are the fallback)

    def to_json(self):
        d = {"UniqueId": self.src, "ConnectionOperator": {"pointwise": "Pointwise", "cross": "CrossProduct",
                                                         "merge": "Pointwise", "broadcast": "CrossProduct",
                                                         "offset": "Pointwise", "group": "Pointwise"}[self.kind],
             "Kind": self.kind, "Port": self.port}
        if self.offset:
            d["Offset"] = self.offset
        if self.merge_sort:
            d["MergeSort"] = True
        if self.group:
            d["GroupSize"] = self.group
        if self.dynamic:
            d["DynamicManager"] = "PartialAggregator"
        return d


@dataclass
class Stage:
    id: int
    name: str
    partitions: int
    inputs: list = field(default_factory=list)
    ops: list = field(default_factory=list)
    out_ports: int = 1
    dtype: object = None
    info: DataSetInfo = field(default_factory=DataSetInfo)
    output: dict | None = None          # {"uri", "delete_if_exists", "temp"} for ToStore stages
    dynamic_manager: str | None = None
    channel_type: str = "DiskFile"
    explain: list = field(default_factory=list)
    gang: bool = False                  # vertices must run together (collective exchange)
    gpu: dict | None = None             # columnar/HIP lowering chosen by the GPU executor

    @property
    def is_output(self) -> bool:
        return self.output is not None

    def describe_ops(self) -> str:
        return " -> ".join(op.get("explain", op["op"]) for op in self.ops)

    def to_json(self):
        return {
            "UniqueId": self.id, "Type": self.ops[0]["op"] if self.ops else "Merge", "Name": self.name,
            "Explain": self.explain + [self.describe_ops()], "Partitions": self.partitions,
            "ChannelType": self.channel_type, "DynamicManager": self.dynamic_manager or "None",
            "Entry": [op["op"] for op in self.ops], "OutputPorts": self.out_ports,
            "Children": [i.to_json() for i in self.inputs],
            "DataSetInfo": self.info.describe(),
            **({"Output": {k: v for k, v in self.output.items() if k in ("uri", "delete_if_exists", "temp")}}
               if self.output else {}),
        }


@dataclass
class Plan:
    stages: list
    outputs: list            # stage ids that write tables (ToStore), in query order
    globals: dict = field(default_factory=dict)

    def stage(self, i) -> Stage:
        return self.stages[i]

    def consumers(self, sid: int) -> list:
        return [s.id for s in self.stages if any(i.src == sid for i in s.inputs)]

    def to_json(self) -> dict:
        return {"Query": {**self.globals, "QueryPlan": [s.to_json() for s in self.stages],
                          "Outputs": self.outputs}}

    def dumps(self) -> str:
        return json.dumps(self.to_json(), indent=1, default=str)

    # reference vertex Type names (DryadLinqQueryNode.QueryNodeType) of the plan's first op
    _XML_TYPE = {"read": "InputTable", "output": "OutputTable", "sort": "OrderBy", "hash_partition": "HashPartition",
                 "range_partition": "RangePartition", "group_partial": "GroupBy", "group_final": "GroupBy",
                 "group_by": "GroupBy", "where": "Where", "select": "Select", "select_many": "SelectMany",
                 "join": "Join", "hash_join": "Join", "group_join": "GroupJoin", "distinct": "Distinct",
                 "union": "Union", "intersect": "Intersect", "except": "Except", "concat": "Concat",
                 "sample": "Dynamic", "separators": "Dynamic", "apply": "Apply", "fork": "Fork",
                 "merge": "Merge", "enumerable": "InputTable", "take": "Take", "skip": "Skip"}

    def to_xml(self) -> str:
        """The plan as the reference's query-plan XML document (DryadLinqQueryGen.cs:837-971,
        DryadLinqQueryNode.cs:769-827): global <Query> properties, then one <Vertex> per stage with
        UniqueId / Type / Name / Explain (CDATA) / Partitions / ChannelType / ConnectionOperator /
        DynamicManager / Entry and <Children> (<Child> UniqueId + AffinityConstraint)."""
        root = ET.Element("Query")
        g = self.globals
        for k in ("DryadLinqVersion", "ClusterName", "MinimumComputeNodes", "MaximumComputeNodes",
                  "IntermediateDataCompression", "EnableSpeculativeDuplication"):
            ET.SubElement(root, k).text = str(g.get(k, ""))
        ET.SubElement(root, "Visualization").text = "none"
        ET.SubElement(root, "QueryName").text = str(g.get("QueryName") or "")
        ET.SubElement(root, "XmlExecHostArgs")
        ET.SubElement(root, "Resources")
        qp = ET.SubElement(root, "QueryPlan")
        cdata = {}
        for st in self.stages:
            v = ET.SubElement(qp, "Vertex")
            ET.SubElement(v, "UniqueId").text = str(st.id)
            first = st.ops[0]["op"] if st.ops else "merge"
            # a stage fusing several operators is the reference's "Super" node
            ET.SubElement(v, "Type").text = "Super" if len(st.ops) > 1 else self._XML_TYPE.get(first, first)
            ET.SubElement(v, "Name").text = st.name
            mark = f"@@CDATA{st.id}@@"
            ET.SubElement(v, "Explain").text = mark
            cdata[mark] = "\n".join(st.explain + [st.describe_ops()])
            ET.SubElement(v, "Partitions").text = str(st.partitions)
            ET.SubElement(v, "ChannelType").text = st.channel_type
            con = st.inputs[0].to_json()["ConnectionOperator"] if st.inputs else "Pointwise"
            ET.SubElement(v, "ConnectionOperator").text = con
            dm = ET.SubElement(v, "DynamicManager")
            ET.SubElement(dm, "Type").text = st.dynamic_manager or "None"
            ET.SubElement(v, "Entry").text = ".".join(op["op"] for op in st.ops)
            if st.output:
                ET.SubElement(v, "StorageSet").text = str(st.output.get("uri", ""))
            ch = ET.SubElement(v, "Children")
            for i in st.inputs:
                c = ET.SubElement(ch, "Child")
                ET.SubElement(c, "UniqueId").text = str(i.src)
                ET.SubElement(c, "AffinityConstraint").text = "UseDefault"
        ET.indent(root)
        text = ET.tostring(root, encoding="unicode")
        for mark, body in cdata.items():
            text = text.replace(mark, "<![CDATA[" + body.replace("]]>", "]]]]><![CDATA[>") + "]]>")
        return '<?xml version="1.0" encoding="utf-8"?>\n' + text + "\n"

    def explain(self) -> str:
        """Human-readable per-stage explanation (reference DryadLinqQueryExplain.cs)."""
        lines = []
        for s in self.stages:
            ins = ", ".join(f"{i.kind}({i.src}" + (f":{i.port}" if i.port else "") + ")" for i in s.inputs) or "-"
            lines.append(f"Stage {s.id} [{s.name}] partitions={s.partitions} inputs={ins}"
                         + (f" ports={s.out_ports}" if s.out_ports != 1 else "")
                         + (f" dynamic={s.dynamic_manager}" if s.dynamic_manager else "")
                         + (" gang" if s.gang else ""))
            for e in s.explain:
                lines.append(f"    {e}")
            for op in s.ops:
                lines.append(f"    {op.get('explain', op['op'])}")
            lines.append(f"    => {s.info.describe()}" + (f" -> {s.output['uri']}" if s.output else ""))
        return "\n".join(lines)
