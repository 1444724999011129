#include "jobgraph.h"

#include <algorithm>
#include <cstdio>
#include <sstream>
#include <stdexcept>

namespace dryad {

const char* vstate_name(VState s) {
  switch (s) {
    case VState::Waiting: return "Waiting";
    case VState::Ready: return "Ready";
    case VState::Running: return "Running";
    case VState::Completed: return "Completed";
    case VState::Failed: return "Failed";
    case VState::Cancelled: return "Cancelled";
  }
  return "?";
}

static std::string jesc(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 8);
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if ((unsigned char)c < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o += c;
        }
    }
  }
  return o;
}

JobGraph::JobGraph(Params p) : p_(p) {
  if (!p_.speculative) {
    // reference: disabling duplication = infinite default threshold and fraction 1.0
    p_.default_outlier_threshold = -1;
    p_.nonparametric_fraction = 1.0;
  }
}

int JobGraph::add_stage(const std::string& name, int partitions, bool speculative, bool is_output) {
  Stage s;
  s.name = name;
  s.partitions = partitions;
  s.speculative = speculative && p_.speculative;
  s.is_output = is_output;
  stages_.push_back(s);
  return (int)stages_.size() - 1;
}

int JobGraph::add_vertex(int stage, int partition) {
  if (stage < 0 || stage >= (int)stages_.size()) throw std::out_of_range("bad stage");
  Vertex v;
  v.id = (int)vertices_.size();
  v.stage = stage;
  v.partition = partition;
  vertices_.push_back(v);
  stages_[stage].vertices.push_back(v.id);
  return v.id;
}

void JobGraph::add_edge(int src, int src_port, int dst, int dst_port) {
  if (src < 0 || dst < 0 || src >= (int)vertices_.size() || dst >= (int)vertices_.size())
    throw std::out_of_range("bad edge");
  Edge e{src, src_port, dst, dst_port};
  edges_.push_back(e);
  int id = (int)edges_.size() - 1;
  vertices_[src].out_edges.push_back(id);
  vertices_[dst].in_edges.push_back(id);
  vertices_[dst].missing_inputs += 1;
}

void JobGraph::set_gang(const std::vector<int>& vs) {
  int g = (int)gangs_.size();
  gangs_.push_back(vs);
  for (int v : vs) vertices_.at(v).gang = g;
}

void JobGraph::set_preferred_workers(int v, const std::vector<int>& w) { vertices_.at(v).preferred_workers = w; }

void JobGraph::event(const std::string& json) { events_.push_back(json); }

std::vector<std::string> JobGraph::drain_events() {
  std::vector<std::string> out;
  out.swap(events_);
  return out;
}

void JobGraph::enqueue(int v, double now, bool duplicate) {
  Vertex& x = vertices_[v];
  Attempt a;
  a.version = x.next_version++;
  a.state = VState::Ready;
  a.queued = now;
  a.duplicate = duplicate;
  x.attempts[a.version] = a;
  x.queued = true;
  ready_.push_back(ReadyItem{v, a.version, duplicate});
  std::ostringstream o;
  o << "{\"ev\":\"vertex\",\"t\":" << now << ",\"vertex\":" << v << ",\"stage\":\"" << jesc(stages_[x.stage].name)
    << "\",\"partition\":" << x.partition << ",\"version\":" << a.version << ",\"state\":\"Ready\""
    << (duplicate ? ",\"duplicate\":true" : "") << "}";
  event(o.str());
}

void JobGraph::start(double now) {
  if (started_) return;
  started_ = true;
  std::ostringstream o;
  o << "{\"ev\":\"job_start\",\"t\":" << now << ",\"vertices\":" << vertices_.size() << ",\"stages\":"
    << stages_.size() << ",\"edges\":" << edges_.size() << "}";
  event(o.str());
  for (auto& v : vertices_)
    if (v.missing_inputs == 0) enqueue(v.id, now, false);
  if (vertices_.empty()) completed_ = 0;
}

std::vector<ReadyItem> JobGraph::take_ready(int max_items, double now) {
  std::vector<ReadyItem> out;
  size_t scan = ready_.size();
  while (!ready_.empty() && (int)out.size() < max_items && scan-- > 0) {
    ReadyItem it = ready_.front();
    ready_.pop_front();
    Vertex& x = vertices_[it.vertex];
    auto f = x.attempts.find(it.version);
    if (f == x.attempts.end() || f->second.state != VState::Ready) continue;
    if (x.completed_version >= 0 || x.missing_inputs > 0 || failed_) {
      f->second.state = VState::Cancelled;
      x.queued = false;
      continue;
    }
    x.queued = false;
    out.push_back(it);
  }
  (void)now;
  return out;
}

void JobGraph::on_running(int v, int version, int worker, double now) {
  Vertex& x = vertices_.at(v);
  auto f = x.attempts.find(version);
  if (f == x.attempts.end()) return;
  // an attempt cancelled meanwhile (gang restart, lost duplicate) stays cancelled
  if (f->second.state == VState::Cancelled || f->second.state == VState::Failed) return;
  f->second.state = VState::Running;
  f->second.worker = worker;
  f->second.start = now;
  stages_[x.stage].stats.started++;
  std::ostringstream o;
  o << "{\"ev\":\"vertex\",\"t\":" << now << ",\"vertex\":" << v << ",\"stage\":\"" << jesc(stages_[x.stage].name)
    << "\",\"partition\":" << x.partition << ",\"version\":" << version << ",\"state\":\"Running\",\"worker\":"
    << worker << "}";
  event(o.str());
}

int JobGraph::running_count() const {
  int n = 0;
  for (auto& v : vertices_)
    for (auto& kv : v.attempts)
      if (kv.second.state == VState::Running) ++n;
  return n;
}

VState JobGraph::state(int v) const {
  const Vertex& x = vertices_.at(v);
  if (x.completed_version >= 0) return VState::Completed;
  bool ready = false;
  for (auto& kv : x.attempts) {
    if (kv.second.state == VState::Running) return VState::Running;
    if (kv.second.state == VState::Ready) ready = true;
  }
  return ready ? VState::Ready : VState::Waiting;
}

void JobGraph::mark_completed_downstream(int v, double now) {
  for (int e : vertices_[v].out_edges) {
    Vertex& d = vertices_[edges_[e].dst];
    d.missing_inputs -= 1;
    if (d.missing_inputs == 0 && d.completed_version < 0 && !d.queued) {
      bool live = false;
      for (auto& kv : d.attempts)
        if (kv.second.state == VState::Running) live = true;
      if (!live) enqueue(d.id, now, false);
    }
  }
}

void JobGraph::reestimate(Stage& s) {
  StageStats& st = s.stats;
  const int n = (int)st.elapsed.size();
  const int need = std::max(2, (int)(s.partitions * 0.5));
  if (n < need) return;
  std::vector<double> e = st.elapsed;
  std::sort(e.begin(), e.end());
  const int idx = (int)((double)st.started * p_.nonparametric_fraction);
  if (idx < n) st.estimate = std::max(e[idx], p_.min_outlier_threshold);
}

double JobGraph::outlier_threshold(int stage) const {
  const Stage& s = stages_.at(stage);
  if (!s.speculative) return -1;
  const double est = s.stats.estimate;
  if (s.partitions <= p_.duplicate_everything_threshold) {
    if (p_.default_outlier_threshold < 0) return est;   // disabled: only a computed estimate
    if (est >= 0 && est < p_.default_outlier_threshold) return est;
    return p_.default_outlier_threshold;
  }
  return est;
}

std::vector<std::pair<int, int>> JobGraph::on_completed(int v, int version, double now, int64_t bytes_read,
                                                        int64_t bytes_written, bool* accepted) {
  std::vector<std::pair<int, int>> cancel;
  Vertex& x = vertices_.at(v);
  auto f = x.attempts.find(version);
  *accepted = false;
  if (f == x.attempts.end() || f->second.state == VState::Cancelled || f->second.state == VState::Failed) return cancel;
  f->second.end = now;
  if (x.completed_version >= 0) {
    f->second.state = VState::Cancelled;   // a duplicate lost the race
    return cancel;
  }
  *accepted = true;
  const bool was_running = f->second.state == VState::Running;
  f->second.state = VState::Completed;
  x.completed_version = version;
  x.bytes_read += bytes_read;
  x.bytes_written += bytes_written;
  completed_++;
  Stage& s = stages_[x.stage];
  s.completed++;
  if (was_running) s.stats.elapsed.push_back(now - f->second.start);
  reestimate(s);
  for (auto& kv : x.attempts) {
    if (kv.first != version && (kv.second.state == VState::Running || kv.second.state == VState::Ready)) {
      if (kv.second.state == VState::Running) cancel.push_back({v, kv.first});
      kv.second.state = VState::Cancelled;
    }
  }
  x.queued = false;
  std::ostringstream o;
  o << "{\"ev\":\"vertex\",\"t\":" << now << ",\"vertex\":" << v << ",\"stage\":\"" << jesc(s.name)
    << "\",\"partition\":" << x.partition << ",\"version\":" << version << ",\"state\":\"Completed\",\"elapsed\":"
    << (was_running ? now - f->second.start : 0.0) << ",\"bytes_read\":" << bytes_read
    << ",\"bytes_written\":" << bytes_written << "}";
  event(o.str());
  mark_completed_downstream(v, now);
  if (done()) {
    std::ostringstream j;
    j << "{\"ev\":\"job_stop\",\"t\":" << now << ",\"status\":\"Success\"}";
    event(j.str());
  }
  return cancel;
}

void JobGraph::invalidate(int v, double now) {
  Vertex& x = vertices_[v];
  if (x.completed_version < 0) return;
  std::ostringstream o;
  o << "{\"ev\":\"vertex\",\"t\":" << now << ",\"vertex\":" << v << ",\"stage\":\"" << jesc(stages_[x.stage].name)
    << "\",\"partition\":" << x.partition << ",\"version\":" << x.completed_version
    << ",\"state\":\"Invalidated\"}";
  event(o.str());
  x.completed_version = -1;
  completed_--;
  stages_[x.stage].completed--;
  for (int e : x.out_edges) vertices_[edges_[e].dst].missing_inputs += 1;
  if (x.missing_inputs == 0 && !x.queued) enqueue(v, now, false);
}

FailureOutcome JobGraph::on_failed(int v, int version, double now, int bad_input_edge, const std::string& err) {
  FailureOutcome out;
  Vertex& x = vertices_.at(v);
  auto f = x.attempts.find(version);
  if (f != x.attempts.end()) {
    if (f->second.state == VState::Cancelled) return out;   // we killed it ourselves
    f->second.state = VState::Failed;
    f->second.end = now;
  }
  {
    std::ostringstream o;
    o << "{\"ev\":\"vertex\",\"t\":" << now << ",\"vertex\":" << v << ",\"stage\":\"" << jesc(stages_[x.stage].name)
      << "\",\"partition\":" << x.partition << ",\"version\":" << version << ",\"state\":\"Failed\",\"error\":\""
      << jesc(err) << "\",\"bad_input\":" << bad_input_edge << "}";
    event(o.str());
  }
  if (x.completed_version >= 0) return out;   // a duplicate already won
  bool other_live = false;
  for (auto& kv : x.attempts)
    if (kv.first != version && (kv.second.state == VState::Running || kv.second.state == VState::Ready))
      other_live = true;
  if (bad_input_edge >= 0 && bad_input_edge < (int)edges_.size() && edges_[bad_input_edge].dst == v) {
    // read error: blame (and re-run) the producer instead of this vertex
    const int src = edges_[bad_input_edge].src;
    out.action = 1;
    out.invalidated_vertex = src;
    invalidate(src, now);
    return out;
  }
  x.failures += 1;
  if (x.failures >= p_.max_failures) {
    std::ostringstream m;
    m << "Graph abort because vertex failed " << x.failures << " times: vertex " << v << " ("
      << stages_[x.stage].name << "[" << x.partition << "]). VERTEX FAILURE DETAILS: " << err;
    abort(m.str());
    out.action = 2;
    out.message = failure_;
    return out;
  }
  if (x.gang >= 0) {
    // restart the whole gang: cancel every live attempt of every member, requeue all
    for (int m : gangs_[x.gang]) {
      Vertex& y = vertices_[m];
      for (auto& kv : y.attempts) {
        if (kv.second.state == VState::Running) {
          out.cancel.push_back({m, kv.first});
          kv.second.state = VState::Cancelled;
        } else if (kv.second.state == VState::Ready) {
          kv.second.state = VState::Cancelled;
        }
      }
      if (y.completed_version >= 0) {
        y.completed_version = -1;
        completed_--;
        stages_[y.stage].completed--;
        for (int e : y.out_edges) vertices_[edges_[e].dst].missing_inputs += 1;
      }
      y.queued = false;
    }
    for (int m : gangs_[x.gang])
      if (vertices_[m].missing_inputs == 0) enqueue(m, now, false);
    out.action = 0;
    return out;
  }
  if (!other_live && x.missing_inputs == 0 && !x.queued) enqueue(v, now, false);
  out.action = 0;
  return out;
}

void JobGraph::on_cancelled(int v, int version, double now) {
  Vertex& x = vertices_.at(v);
  auto f = x.attempts.find(version);
  if (f == x.attempts.end()) return;
  f->second.state = VState::Cancelled;
  f->second.end = now;
}

std::vector<ReadyItem> JobGraph::check_duplicates(double now) {
  std::vector<ReadyItem> out;
  if (failed_) return out;
  for (int si = 0; si < (int)stages_.size(); ++si) {
    const double thr = outlier_threshold(si);
    if (thr < 0) continue;
    for (int v : stages_[si].vertices) {
      Vertex& x = vertices_[v];
      if (x.completed_version >= 0 || x.queued || x.gang >= 0) continue;
      int live = 0;
      double start = 0;
      bool has_dup = false;
      for (auto& kv : x.attempts) {
        if (kv.second.state == VState::Running) {
          ++live;
          start = kv.second.start;
          has_dup |= kv.second.duplicate;
        }
      }
      if (live == 1 && !has_dup && start + thr < now) {
        enqueue(v, now, true);
        out.push_back(ready_.back());
      }
    }
  }
  return out;
}

void JobGraph::abort(const std::string& why) {
  if (failed_) return;
  failed_ = true;
  failure_ = why;
  ready_.clear();
  std::ostringstream j;
  j << "{\"ev\":\"job_stop\",\"status\":\"Failure\",\"error\":\"" << jesc(why) << "\"}";
  event(j.str());
}

std::string JobGraph::topology_json() const {
  std::ostringstream o;
  o << "{\"stages\":[";
  for (size_t i = 0; i < stages_.size(); ++i) {
    if (i) o << ",";
    o << "{\"id\":" << i << ",\"name\":\"" << jesc(stages_[i].name) << "\",\"partitions\":" << stages_[i].partitions
      << ",\"vertices\":[";
    for (size_t k = 0; k < stages_[i].vertices.size(); ++k) o << (k ? "," : "") << stages_[i].vertices[k];
    o << "]}";
  }
  o << "],\"edges\":[";
  for (size_t i = 0; i < edges_.size(); ++i) {
    if (i) o << ",";
    o << "[" << edges_[i].src << "," << edges_[i].src_port << "," << edges_[i].dst << "," << edges_[i].dst_port << "]";
  }
  o << "]}";
  return o.str();
}

std::string JobGraph::statistics_json() const {
  std::ostringstream o;
  o << "{\"stages\":[";
  for (size_t i = 0; i < stages_.size(); ++i) {
    const Stage& s = stages_[i];
    double tot = 0, mx = 0;
    for (double e : s.stats.elapsed) {
      tot += e;
      mx = std::max(mx, e);
    }
    int64_t br = 0, bw = 0;
    int versions = 0, failures = 0;
    for (int v : s.vertices) {
      br += vertices_[v].bytes_read;
      bw += vertices_[v].bytes_written;
      versions += vertices_[v].next_version;
      failures += vertices_[v].failures;
    }
    if (i) o << ",";
    o << "{\"name\":\"" << jesc(s.name) << "\",\"partitions\":" << s.partitions << ",\"completed\":" << s.completed
      << ",\"executions\":" << versions << ",\"failures\":" << failures << ",\"mean_s\":"
      << (s.stats.elapsed.empty() ? 0.0 : tot / s.stats.elapsed.size()) << ",\"max_s\":" << mx
      << ",\"outlier_threshold_s\":" << outlier_threshold((int)i) << ",\"bytes_read\":" << br
      << ",\"bytes_written\":" << bw << "}";
  }
  o << "]}";
  return o.str();
}

// ------------------------------------------------------------------------------------------
Scheduler::Scheduler(int workers, double locality_delay)
    : busy_(workers, false), alive_(workers, true), delay_(locality_delay) {}

int Scheduler::add_worker() {
  busy_.push_back(false);
  alive_.push_back(true);
  return (int)busy_.size() - 1;
}

void Scheduler::set_alive(int w, bool alive) {
  alive_.at(w) = alive;
  if (!alive) busy_.at(w) = false;
}

void Scheduler::release(int w) { busy_.at(w) = false; }

bool Scheduler::idle(int w) const { return alive_.at(w) && !busy_.at(w); }

int Scheduler::idle_count() const {
  int n = 0;
  for (size_t i = 0; i < busy_.size(); ++i)
    if (alive_[i] && !busy_[i]) ++n;
  return n;
}

void Scheduler::set_busy(int w) { busy_.at(w) = true; }

int Scheduler::place(const std::vector<int>& preferred, double waited) {
  for (int w : preferred)
    if (w >= 0 && w < (int)busy_.size() && idle(w)) return w;
  if (!preferred.empty() && waited < delay_) return -1;
  for (int w = 0; w < (int)busy_.size(); ++w)
    if (idle(w)) return w;
  return -1;
}

}  // namespace dryad
