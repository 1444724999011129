// Dryad-AMD job manager core: the stage/vertex DAG state machine.
//
// Reference behaviour reproduced (GraphManager/):
//   * vertices are (stage, partition); every execution attempt is a numbered *version*
//     (DrActiveVertex::InstantiateVersion, GraphManager/vertex/DrVertex.cpp:531-562)
//   * a vertex becomes ready when every upstream vertex has a completed version
//     (ReactToUpStreamCompletedVertex, DrVertex.cpp:860)
//   * failure policy (DrGraph::ReportFailure, GraphManager/vertex/DrGraph.cpp:392-456): a failure
//     blamed on an input channel invalidates the upstream vertex's completed version, which is
//     re-executed; any other failure counts against the vertex and the job aborts after
//     max_failures (6, DrGraphParameters.cpp:52)
//   * speculative duplication (DrManagerBase::CheckForDuplicates, stagemanager/DrDefaultManager.cpp:
//     664-714): once the non-parametric outlier threshold of a stage is known, a vertex running
//     longer than it gets a duplicate version; the first version to complete wins and the others
//     are cancelled (DrStageStatistics::GetOutlierThreshold, DrStageStatistics.cpp:93-111)
//   * gangs (DrGang, DrCohort.cpp:852): vertices that must run together (on MI355X: the members of
//     one RCCL collective exchange); any member failure cancels and restarts the whole gang
//   * job event log in the Calypso vocabulary (DrCalypsoReporting.cpp) as JSON lines
#pragma once
#include <cstdint>
#include <deque>
#include <map>
#include <set>
#include <string>
#include <vector>

namespace dryad {

enum class VState : int { Waiting = 0, Ready = 1, Running = 2, Completed = 3, Failed = 4, Cancelled = 5 };

const char* vstate_name(VState s);

struct Edge {
  int src;
  int src_port;
  int dst;
  int dst_port;
};

struct Attempt {
  int version = 0;
  VState state = VState::Ready;
  int worker = -1;
  double queued = 0, start = 0, end = 0;
  bool duplicate = false;
};

struct Vertex {
  int id = 0;
  int stage = 0;
  int partition = 0;
  std::vector<int> in_edges, out_edges;
  int completed_version = -1;
  int next_version = 0;
  int failures = 0;
  int missing_inputs = 0;   // upstream vertices without a completed version
  bool queued = false;      // an attempt is in the ready queue
  int gang = -1;
  std::map<int, Attempt> attempts;  // version -> attempt
  std::vector<int> preferred_workers;
  int64_t bytes_read = 0, bytes_written = 0;
};

struct StageStats {
  std::vector<double> elapsed;   // completed execution times (seconds)
  int started = 0;
  double estimate = -1;          // non-parametric outlier estimate, <0 = unknown
};

struct Stage {
  std::string name;
  int partitions = 0;
  std::vector<int> vertices;
  bool speculative = true;
  bool is_output = false;
  int completed = 0;
  StageStats stats;
};

struct Params {
  int max_failures = 6;                 // DrGraphParameters m_maxActiveFailureCount
  int duplicate_everything_threshold = 10;
  double default_outlier_threshold = 600.0;   // 10 min
  double min_outlier_threshold = 10.0;        // 10 s
  double nonparametric_fraction = 0.5;
  bool speculative = true;
};

struct ReadyItem {
  int vertex;
  int version;
  bool duplicate;
};

struct FailureOutcome {
  // 0 = retry scheduled, 1 = upstream invalidated (vertex waits), 2 = job aborted
  int action = 0;
  int invalidated_vertex = -1;
  std::vector<std::pair<int, int>> cancel;  // (vertex, version) attempts to kill (gang restart)
  std::string message;
};

class JobGraph {
 public:
  explicit JobGraph(Params p = Params());

  int add_stage(const std::string& name, int partitions, bool speculative, bool is_output);
  int add_vertex(int stage, int partition);
  void add_edge(int src, int src_port, int dst, int dst_port);
  void set_gang(const std::vector<int>& vertices);
  void set_preferred_workers(int vertex, const std::vector<int>& workers);

  void start(double now);
  std::vector<ReadyItem> take_ready(int max_items, double now);
  void on_running(int vertex, int version, int worker, double now);
  // returns (vertex,version) attempts that became redundant and should be cancelled; the bool
  // `accepted` says whether this completion was the winning one.
  std::vector<std::pair<int, int>> on_completed(int vertex, int version, double now, int64_t bytes_read,
                                                int64_t bytes_written, bool* accepted);
  FailureOutcome on_failed(int vertex, int version, double now, int bad_input_edge, const std::string& err);
  void on_cancelled(int vertex, int version, double now);
  std::vector<ReadyItem> check_duplicates(double now);
  void abort(const std::string& why);

  bool done() const { return completed_ == (int)vertices_.size(); }
  bool failed() const { return failed_; }
  const std::string& failure() const { return failure_; }
  int completed_version(int v) const { return vertices_.at(v).completed_version; }
  int vertex_count() const { return (int)vertices_.size(); }
  int stage_count() const { return (int)stages_.size(); }
  int ready_count() const { return (int)ready_.size(); }
  int running_count() const;
  VState state(int v) const;
  const Vertex& vertex(int v) const { return vertices_.at(v); }
  const Stage& stage(int s) const { return stages_.at(s); }
  const std::vector<Edge>& edges() const { return edges_; }
  double outlier_threshold(int stage) const;
  std::vector<std::string> drain_events();
  std::string topology_json() const;
  std::string statistics_json() const;
  // Append one JSON event line (the executor's own events: gang relaunch, resumed stages).
  void event(const std::string& json);

 private:
  void enqueue(int v, double now, bool duplicate);
  void mark_completed_downstream(int v, double now);
  void invalidate(int v, double now);
  void reestimate(Stage& s);

  Params p_;
  std::vector<Stage> stages_;
  std::vector<Vertex> vertices_;
  std::vector<Edge> edges_;
  std::deque<ReadyItem> ready_;
  std::vector<std::vector<int>> gangs_;
  int completed_ = 0;
  bool failed_ = false;
  bool started_ = false;
  std::string failure_;
  std::vector<std::string> events_;
};

// Worker-slot scheduler with locality preference and delay scheduling (LocalScheduler.cs:52-53,
// 132-268: computer queue, then rack after 1 s, cluster after 2 s).  Here: a vertex first waits up
// to `locality_delay` seconds for one of its preferred workers, then takes any idle one.
class Scheduler {
 public:
  explicit Scheduler(int workers, double locality_delay = 0.0);
  int add_worker();
  void set_alive(int w, bool alive);
  void release(int w);
  bool idle(int w) const;
  int idle_count() const;
  // choose a worker for the item; -1 = none now (keep it pending)
  int place(const std::vector<int>& preferred, double waited);
  void set_busy(int w);
  int size() const { return (int)busy_.size(); }

 private:
  std::vector<bool> busy_, alive_;
  double delay_;
};

}  // namespace dryad
