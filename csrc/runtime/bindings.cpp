// pybind11 module `_dryad_native`: the C++ runtime exposed to the Python planner/executors.
#include <cstring>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "codec.h"
#include "fifo.h"
#include "jobgraph.h"
#include "partreader.h"
#include "partwriter.h"
#include "pump.h"
#include "workqueue.h"

namespace py = pybind11;
using namespace dryad;

namespace {

std::vector<FieldKind> to_schema(const std::vector<int>& s) {
  std::vector<FieldKind> k;
  k.reserve(s.size());
  for (int x : s) {
    if (x < 0 || x > (int)FieldKind::String) throw std::invalid_argument("bad field kind");
    k.push_back((FieldKind)x);
  }
  return k;
}

py::bytes as_bytes(const std::vector<uint8_t>& v) { return py::bytes(reinterpret_cast<const char*>(v.data()), v.size()); }

// decode a record stream into a list of columns: numpy uint8 buffers for fixed fields (caller
// views them with the right dtype) and (offsets int64, data uint8) tuples for strings.
py::tuple py_decode(py::buffer buf, const std::vector<int>& schema_codes) {
  py::buffer_info bi = buf.request();
  const auto schema = to_schema(schema_codes);
  std::vector<std::vector<uint8_t>> fixed;
  std::vector<StringColumn> strings;
  size_t n;
  {
    py::gil_scoped_release nogil;
    n = decode_records(reinterpret_cast<const uint8_t*>(bi.ptr), (size_t)bi.size * bi.itemsize, schema, fixed,
                       strings);
  }
  py::list cols;
  for (size_t f = 0; f < schema.size(); ++f) {
    if (schema[f] == FieldKind::String) {
      auto& sc = strings[f];
      py::array_t<int64_t> off(sc.offsets.size());
      std::memcpy(off.mutable_data(), sc.offsets.data(), sc.offsets.size() * sizeof(int64_t));
      py::array_t<uint8_t> dat(sc.data.size());
      if (!sc.data.empty()) std::memcpy(dat.mutable_data(), sc.data.data(), sc.data.size());
      cols.append(py::make_tuple(off, dat));
    } else {
      py::array_t<uint8_t> a(fixed[f].size());
      if (!fixed[f].empty()) std::memcpy(a.mutable_data(), fixed[f].data(), fixed[f].size());
      cols.append(a);
    }
  }
  return py::make_tuple(n, cols);
}

py::bytes py_encode(size_t n, const std::vector<int>& schema_codes, py::list cols) {
  const auto schema = to_schema(schema_codes);
  if ((size_t)py::len(cols) != schema.size()) throw std::invalid_argument("column count != schema");
  std::vector<const uint8_t*> fixed(schema.size(), nullptr);
  std::vector<StringColumn> owned(schema.size());
  std::vector<const StringColumn*> strings(schema.size(), nullptr);
  std::vector<py::buffer_info> keep;
  for (size_t f = 0; f < schema.size(); ++f) {
    if (schema[f] == FieldKind::String) {
      py::tuple t = cols[f].cast<py::tuple>();
      auto off = t[0].cast<py::array_t<int64_t, py::array::c_style | py::array::forcecast>>();
      auto dat = t[1].cast<py::array_t<uint8_t, py::array::c_style | py::array::forcecast>>();
      owned[f].offsets.assign(off.data(), off.data() + off.size());
      owned[f].data.assign(dat.data(), dat.data() + dat.size());
      if (owned[f].offsets.size() < n + 1) throw std::invalid_argument("string offsets too short");
      strings[f] = &owned[f];
    } else {
      py::buffer b = cols[f].cast<py::buffer>();
      keep.push_back(b.request());
      const auto& bi = keep.back();
      if ((size_t)(bi.size * bi.itemsize) < n * (size_t)field_width(schema[f]))
        throw std::invalid_argument("fixed column too short");
      fixed[f] = reinterpret_cast<const uint8_t*>(bi.ptr);
    }
  }
  std::vector<uint8_t> out;
  {
    py::gil_scoped_release nogil;
    out = encode_records(n, schema, fixed, strings);
  }
  return as_bytes(out);
}

py::tuple py_split_lines(py::buffer buf) {
  py::buffer_info bi = buf.request();
  std::vector<int64_t> st, en;
  {
    py::gil_scoped_release nogil;
    split_lines(reinterpret_cast<const uint8_t*>(bi.ptr), (size_t)bi.size * bi.itemsize, st, en);
  }
  py::array_t<int64_t> a(st.size()), b(en.size());
  if (!st.empty()) {
    std::memcpy(a.mutable_data(), st.data(), st.size() * 8);
    std::memcpy(b.mutable_data(), en.data(), en.size() * 8);
  }
  return py::make_tuple(a, b);
}

struct PyReadBatch {
  std::shared_ptr<ReadBatch> b;
  py::bytes get(size_t i) {
    if (i >= b->paths.size()) throw std::out_of_range("read batch index");
    {
      py::gil_scoped_release nogil;
      wait_read(*b, i);
    }
    if (!b->errors[i].empty()) throw std::runtime_error(b->errors[i]);
    return py::bytes(b->data[i]);
  }
  size_t size() const { return b->paths.size(); }
};

}  // namespace

PYBIND11_MODULE(_dryad_native, m) {
  m.doc() = "Dryad-AMD native runtime: job manager, scheduler, codec, fingerprints, work queue";

  py::enum_<VState>(m, "VState")
      .value("Waiting", VState::Waiting).value("Ready", VState::Ready).value("Running", VState::Running)
      .value("Completed", VState::Completed).value("Failed", VState::Failed).value("Cancelled", VState::Cancelled);

  py::class_<Params>(m, "Params")
      .def(py::init<>())
      .def_readwrite("max_failures", &Params::max_failures)
      .def_readwrite("duplicate_everything_threshold", &Params::duplicate_everything_threshold)
      .def_readwrite("default_outlier_threshold", &Params::default_outlier_threshold)
      .def_readwrite("min_outlier_threshold", &Params::min_outlier_threshold)
      .def_readwrite("nonparametric_fraction", &Params::nonparametric_fraction)
      .def_readwrite("speculative", &Params::speculative);

  py::class_<ReadyItem>(m, "ReadyItem")
      .def_readonly("vertex", &ReadyItem::vertex)
      .def_readonly("version", &ReadyItem::version)
      .def_readonly("duplicate", &ReadyItem::duplicate)
      .def("__repr__", [](const ReadyItem& r) {
        return "<ReadyItem v" + std::to_string(r.vertex) + "." + std::to_string(r.version) + (r.duplicate ? " dup>" : ">");
      });

  py::class_<FailureOutcome>(m, "FailureOutcome")
      .def_readonly("action", &FailureOutcome::action)
      .def_readonly("invalidated_vertex", &FailureOutcome::invalidated_vertex)
      .def_readonly("cancel", &FailureOutcome::cancel)
      .def_readonly("message", &FailureOutcome::message);

  py::class_<JobGraph>(m, "JobGraph")
      .def(py::init<Params>(), py::arg("params") = Params())
      .def("add_stage", &JobGraph::add_stage, py::arg("name"), py::arg("partitions"), py::arg("speculative") = true,
           py::arg("is_output") = false)
      .def("add_vertex", &JobGraph::add_vertex)
      .def("add_edge", &JobGraph::add_edge)
      .def("set_gang", &JobGraph::set_gang)
      .def("set_preferred_workers", &JobGraph::set_preferred_workers)
      .def("start", &JobGraph::start)
      .def("take_ready", &JobGraph::take_ready)
      .def("on_running", &JobGraph::on_running)
      .def("on_completed",
           [](JobGraph& g, int v, int ver, double now, int64_t br, int64_t bw) {
             bool acc = false;
             auto c = g.on_completed(v, ver, now, br, bw, &acc);
             return py::make_tuple(acc, c);
           },
           py::arg("vertex"), py::arg("version"), py::arg("now"), py::arg("bytes_read") = 0,
           py::arg("bytes_written") = 0)
      .def("on_failed", &JobGraph::on_failed, py::arg("vertex"), py::arg("version"), py::arg("now"),
           py::arg("bad_input_edge") = -1, py::arg("error") = "")
      .def("on_cancelled", &JobGraph::on_cancelled)
      .def("check_duplicates", &JobGraph::check_duplicates)
      .def("abort", &JobGraph::abort)
      .def("done", &JobGraph::done)
      .def("failed", &JobGraph::failed)
      .def("failure", &JobGraph::failure)
      .def("completed_version", &JobGraph::completed_version)
      .def("vertex_count", &JobGraph::vertex_count)
      .def("stage_count", &JobGraph::stage_count)
      .def("ready_count", &JobGraph::ready_count)
      .def("running_count", &JobGraph::running_count)
      .def("state", &JobGraph::state)
      .def("failures", [](const JobGraph& g, int v) { return g.vertex(v).failures; })
      .def("versions", [](const JobGraph& g, int v) { return g.vertex(v).next_version; })
      .def("vertex_stage", [](const JobGraph& g, int v) { return g.vertex(v).stage; })
      .def("vertex_partition", [](const JobGraph& g, int v) { return g.vertex(v).partition; })
      .def("in_edges", [](const JobGraph& g, int v) { return g.vertex(v).in_edges; })
      .def("edge", [](const JobGraph& g, int e) {
        const Edge& x = g.edges().at(e);
        return py::make_tuple(x.src, x.src_port, x.dst, x.dst_port);
      })
      .def("preferred_workers", [](const JobGraph& g, int v) { return g.vertex(v).preferred_workers; })
      .def("outlier_threshold", &JobGraph::outlier_threshold)
      .def("drain_events", &JobGraph::drain_events)
      .def("event", &JobGraph::event, "append a JSON event line (executor-side events: gang relaunch, resume)")
      .def("topology_json", &JobGraph::topology_json)
      .def("statistics_json", &JobGraph::statistics_json);

  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<int, double>(), py::arg("workers"), py::arg("locality_delay") = 0.0)
      .def("add_worker", &Scheduler::add_worker)
      .def("set_alive", &Scheduler::set_alive)
      .def("release", &Scheduler::release)
      .def("idle", &Scheduler::idle)
      .def("idle_count", &Scheduler::idle_count)
      .def("place", &Scheduler::place)
      .def("set_busy", &Scheduler::set_busy)
      .def("size", &Scheduler::size);

  m.def("decode_records", &py_decode, "record stream -> (n, columns)");
  m.def("encode_records", &py_encode, "columns -> record stream");
  m.def("split_lines", &py_split_lines);
  m.def("lines_to_records", [](py::buffer buf) {
    py::buffer_info bi = buf.request();
    std::vector<uint8_t> out;
    {
      py::gil_scoped_release nogil;
      out = lines_to_records(reinterpret_cast<const uint8_t*>(bi.ptr), (size_t)bi.size * bi.itemsize);
    }
    return as_bytes(out);
  });
  m.def("utf16_units", [](py::bytes b) {
    std::string s = b;
    return utf16_units(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });

  py::class_<Rabin64>(m, "Rabin64")
      .def(py::init<uint64_t>(), py::arg("poly") = 0x911498ae0e66bad6ull)
      .def("empty", &Rabin64::empty)
      .def("extend",
           [](const Rabin64& r, uint64_t fp, py::buffer b) {
             py::buffer_info bi = b.request();
             return r.extend(fp, reinterpret_cast<const uint8_t*>(bi.ptr), (size_t)bi.size * bi.itemsize);
           })
      .def("extend_u16", &Rabin64::extend_u16)
      .def("extend_u32", &Rabin64::extend_u32)
      .def("extend_u64", &Rabin64::extend_u64)
      .def("table", [](const Rabin64& r, int b) {
        py::array_t<uint64_t> a(256);
        std::memcpy(a.mutable_data(), r.table(b), 256 * 8);
        return a;
      });

  py::class_<WorkQueue>(m, "WorkQueue").def(py::init<int>()).def("threads", &WorkQueue::threads).def("drain", [](WorkQueue& q) {
    py::gil_scoped_release nogil;
    q.drain();
  });
  py::class_<PyReadBatch>(m, "ReadBatch").def("get", &PyReadBatch::get).def("__len__", &PyReadBatch::size);
  m.def("read_files_async", [](WorkQueue& q, const std::vector<std::string>& paths) {
    return PyReadBatch{read_files_async(q, paths)};
  });
  m.def("scan_record_blocks", [](py::buffer buf, const std::vector<int>& schema_codes, size_t block) {
    py::buffer_info bi = buf.request();
    const auto schema = to_schema(schema_codes);
    std::vector<int64_t> offs;
    size_t n;
    {
      py::gil_scoped_release nogil;
      n = scan_record_blocks(reinterpret_cast<const uint8_t*>(bi.ptr), (size_t)bi.size * bi.itemsize, schema, block,
                             offs);
    }
    py::array_t<int64_t> a(offs.size());
    if (!offs.empty()) std::memcpy(a.mutable_data(), offs.data(), offs.size() * sizeof(int64_t));
    return py::make_tuple(n, a);
  });
  // ChunkReader: file -> ring of caller-owned (pinned) host buffers, several reader threads.
  py::class_<ChunkReader>(m, "ChunkReader")
      .def(py::init<const std::string&, int64_t, int64_t, int64_t, const std::vector<std::pair<uint64_t, int64_t>>&,
                    int>(),
           py::arg("path"), py::arg("offset"), py::arg("length"), py::arg("chunk_bytes"), py::arg("buffers"),
           py::arg("threads"))
      .def("size", &ChunkReader::size)
      .def("chunks", &ChunkReader::chunks)
      .def("next", [](ChunkReader& r, int64_t timeout_ms) -> py::object {
        ReadyChunk c;
        bool more;
        {
          py::gil_scoped_release nogil;
          more = r.next(&c, timeout_ms);
        }
        if (!more) {
          const std::string e = r.error();
          if (!e.empty()) throw std::runtime_error("ChunkReader: " + e);
          return py::none();
        }
        return py::make_tuple(c.slot, c.chunk, c.bytes);
      }, py::arg("timeout_ms") = -1)
      .def("release", &ChunkReader::release)
      .def("error", &ChunkReader::error)
      .def("stop", [](ChunkReader& r) {
        py::gil_scoped_release nogil;
        r.stop();
      });
  // ChunkWriter: ring of caller-owned (pinned) host buffers -> file, several writer threads.
  py::class_<ChunkWriter>(m, "ChunkWriter")
      .def(py::init<const std::string&, const std::vector<uint64_t>&, int, int64_t, bool>(), py::arg("path"),
           py::arg("buffers"), py::arg("threads"), py::arg("extend_bytes") = (int64_t)(256ll << 20),
           py::arg("mapped") = false)
      .def(py::init<const std::vector<std::string>&, const std::vector<uint64_t>&, int, int64_t, bool>(),
           py::arg("paths"), py::arg("buffers"), py::arg("threads"), py::arg("extend_bytes") = (int64_t)(256ll << 20),
           py::arg("reuse") = false)
      .def("acquire", [](ChunkWriter& w) {
        int s;
        {
          py::gil_scoped_release nogil;
          s = w.acquire();
        }
        if (s < 0) throw std::runtime_error("ChunkWriter: " + w.error());
        return s;
      })
      .def("submit", &ChunkWriter::submit, py::arg("slot"), py::arg("offset"), py::arg("bytes"), py::arg("file") = 0)
      .def("finish", [](ChunkWriter& w, int64_t size) {
        py::gil_scoped_release nogil;
        return w.finish(size);
      })
      .def("finish_all", [](ChunkWriter& w, const std::vector<int64_t>& sizes) {
        py::gil_scoped_release nogil;
        return w.finish_all(sizes);
      })
      .def("error", &ChunkWriter::error)
      .def("abort", [](ChunkWriter& w) {
        py::gil_scoped_release nogil;
        w.abort();
      });
  m.def("write_file_atomic", [](const std::string& path, py::buffer b) {
    py::buffer_info bi = b.request();
    py::gil_scoped_release nogil;
    write_file_atomic(path, reinterpret_cast<const uint8_t*>(bi.ptr), (size_t)bi.size * bi.itemsize);
  });

  // FIFO channel (C-5).  put/get return a status code (0 ok, 1 timeout, 2 closed, 3 aborted);
  // both release the GIL while they wait so producer and consumer threads run concurrently.
  py::class_<BlockFifo>(m, "BlockFifo")
      .def(py::init<uint64_t>(), py::arg("capacity_bytes"))
      .def("put", [](BlockFifo& f, py::buffer b, int64_t timeout_ms) {
            py::buffer_info bi = b.request();
            const auto* p = reinterpret_cast<const uint8_t*>(bi.ptr);
            BlockFifo::Block blk(p, p + (size_t)bi.size * bi.itemsize);
            py::gil_scoped_release nogil;
            return (int)f.put(std::move(blk), timeout_ms);
          }, py::arg("block"), py::arg("timeout_ms") = -1)
      .def("get", [](BlockFifo& f, int64_t timeout_ms) -> py::tuple {
            BlockFifo::Block blk;
            BlockFifo::Status st;
            {
              py::gil_scoped_release nogil;
              st = f.get(blk, timeout_ms);
            }
            if (st != BlockFifo::Status::Ok) return py::make_tuple((int)st, py::none());
            return py::make_tuple(0, as_bytes(blk));
          }, py::arg("timeout_ms") = -1)
      .def("close", &BlockFifo::close)
      .def("abort", &BlockFifo::abort)
      .def("error", &BlockFifo::error)
      .def("queued_bytes", &BlockFifo::queued_bytes)
      .def("queued_blocks", &BlockFifo::queued_blocks)
      .def("peak_bytes", &BlockFifo::peak_bytes)
      .def("blocks_written", &BlockFifo::blocks_written)
      .def("capacity", &BlockFifo::capacity)
      .def("closed", &BlockFifo::closed);

  // Job manager event pump (G-10): wait() releases the GIL until a message or a timer is due.
  py::class_<MessagePump>(m, "MessagePump")
      .def(py::init<>())
      .def("post", &MessagePump::post, py::arg("kind"), py::arg("payload") = 0)
      .def("post_after", &MessagePump::post_after, py::arg("delay_ms"), py::arg("kind"), py::arg("payload") = 0)
      .def("wait", [](MessagePump& p, int64_t timeout_ms) {
            std::vector<MessagePump::Message> got;
            {
              py::gil_scoped_release nogil;
              got = p.wait(timeout_ms);
            }
            py::list out;
            for (auto& x : got) out.append(py::make_tuple(x.kind, x.payload));
            return out;
          }, py::arg("timeout_ms") = -1)
      .def("close", &MessagePump::close)
      .def("pending", &MessagePump::pending)
      .def("posted", &MessagePump::posted)
      .def("delivered", &MessagePump::delivered);
}
