// dryad-launch: start one worker process per GPU of the local node (reference A-7 job
// submission / H-3 ProcessService: LocalJobSubmission.cs starts the graph manager and a vertex
// host per computer; here every rank is a peer SPMD process over RCCL).
//
//   dryad-launch --gpus N [--master-port P] [--log-dir DIR] [--grace-seconds S]
//                [--max-restarts K] [--checkpoint-dir DIR] -- prog args...
//
// Each child gets RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
// MASTER_PORT (the torch.distributed env:// contract) and runs in its own process group.  The
// launcher waits for all ranks; the first rank that fails (non-zero exit or signal) makes it
// SIGTERM the others (SIGKILL after the grace period) so a dead rank never leaves the rest hung
// in a collective — the gang-failure rule of DrGang/DrCohort.
//
// Gang relaunch (--max-restarts K > 0): when the first failure is a LOST process (a rank killed by
// a signal, or one that exits with EX_TEMPFAIL = 75 to ask for it), the whole gang is stopped and
// a fresh gang of NEW child processes is started, up to K times: epoch e gets DRYAD_GANG_EPOCH=e,
// DRYAD_GANG_RESTARTS=K, DRYAD_CHECKPOINT_DIR (the persisted stage outputs it resumes from,
// runtime/checkpoint.py) and MASTER_PORT = P + e (a fresh rendezvous).  The checkpoint directory
// is launcher-owned: <--checkpoint-dir>/dryad-ckpt-<launcher pid>, created at start and removed
// when the launcher exits; nothing else under --checkpoint-dir is ever touched.  Without
// --checkpoint-dir a relaunching launcher (--max-restarts > 0) uses /dev/shm (host memory that
// outlives the ranks; the native part writer fills it at page-cache speed).  Nothing is ever re-exec'd
// in place: a process that initialised the GPU only exits.  A rank that fails with an ordinary
// error code (a deterministic job failure) ends the job as before.  The reference re-executes a
// failed vertex process from its persisted inputs the same way (DrVertex.cpp:1042-1171,
// DrGraph.cpp:392-456).  Every relaunch is one JSON line in <log-dir>/launcher.jsonl.
// Exit status = the last gang's first failure (0 when a gang completed).
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fcntl.h>
#include <ftw.h>
#include <string>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>
#include <vector>

namespace {

std::vector<pid_t> g_children;
volatile sig_atomic_t g_stop = 0;
constexpr int kTempFail = 75;          // EX_TEMPFAIL: "relaunch me"

void on_signal(int sig) {
  g_stop = sig;
}

void kill_all(int sig) {
  for (pid_t p : g_children)
    if (p > 0) kill(-p, sig);
}

int usage() {
  std::fprintf(stderr,
               "usage: dryad-launch --gpus N [--master-port P] [--log-dir DIR] [--grace-seconds S] "
               "[--max-restarts K] [--checkpoint-dir DIR] -- prog args...\n");
  return 2;
}

struct GangResult {
  int code = 0;          // first failure's status (128 + signal for a signal death)
  int rank = -1;
  bool lost = false;     // the first failure was a lost process (signal, or EX_TEMPFAIL)
};

struct Options {
  int n = 1, port = 29511, grace = 10, max_restarts = 0;
  std::string log_dir, ckpt_dir;     // ckpt_dir: the launcher-owned subdirectory (see above)
  char** prog = nullptr;
};

GangResult run_gang(const Options& o, int epoch, const std::string& reason) {
  g_children.assign(o.n, -1);
  for (int r = 0; r < o.n; ++r) {
    pid_t pid = fork();
    if (pid < 0) {
      std::perror("fork");
      kill_all(SIGTERM);
      GangResult g;
      g.code = 1;
      return g;
    }
    if (pid == 0) {
      setpgid(0, 0);
      const std::string rs = std::to_string(r), ns = std::to_string(o.n), ps = std::to_string(o.port + epoch);
      setenv("RANK", rs.c_str(), 1);
      setenv("LOCAL_RANK", rs.c_str(), 1);
      setenv("WORLD_SIZE", ns.c_str(), 1);
      setenv("LOCAL_WORLD_SIZE", ns.c_str(), 1);
      setenv("GROUP_RANK", "0", 1);
      setenv("MASTER_ADDR", "127.0.0.1", 1);
      setenv("MASTER_PORT", ps.c_str(), 1);
      setenv("DRYAD_GANG_EPOCH", std::to_string(epoch).c_str(), 1);
      setenv("DRYAD_GANG_RESTARTS", std::to_string(o.max_restarts).c_str(), 1);
      if (!reason.empty()) setenv("DRYAD_GANG_RELAUNCH_REASON", reason.c_str(), 1);
      if (!o.ckpt_dir.empty()) setenv("DRYAD_CHECKPOINT_DIR", o.ckpt_dir.c_str(), 1);
      if (!getenv("HSA_ENABLE_IPC_MODE_LEGACY")) setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0", 1);
      if (!o.log_dir.empty()) {
        const std::string path = o.log_dir + "/rank" + rs + (epoch ? ".e" + std::to_string(epoch) : "") + ".log";
        int fd = open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0644);
        if (fd >= 0) {
          dup2(fd, 1);
          dup2(fd, 2);
          close(fd);
        }
      }
      execvp(o.prog[0], o.prog);
      std::perror("execvp");
      _exit(127);
    }
    setpgid(pid, pid);
    g_children[r] = pid;
  }

  GangResult res;
  int alive = o.n;
  time_t kill_deadline = 0;
  while (alive > 0) {
    int status = 0;
    pid_t pid = waitpid(-1, &status, 0);
    if (pid < 0) {
      if (g_stop) {
        kill_all(SIGTERM);
        g_stop = 0;
        if (!kill_deadline) kill_deadline = time(nullptr) + o.grace;
        if (res.rank < 0) {       // the launcher itself was stopped: no relaunch
          res.code = 128 + SIGTERM;
          res.rank = o.n;
        }
        continue;
      }
      if (kill_deadline && time(nullptr) > kill_deadline) kill_all(SIGKILL);
      continue;
    }
    int rank = -1;
    for (int r = 0; r < o.n; ++r)
      if (g_children[r] == pid) rank = r;
    if (rank < 0) {
      if (kill_deadline && time(nullptr) > kill_deadline) kill_all(SIGKILL);
      continue;               // the grace-period timer (below)
    }
    g_children[rank] = -1;
    --alive;
    const bool signaled = WIFSIGNALED(status);
    const int code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + WTERMSIG(status);
    std::fprintf(stderr, "[dryad-launch] epoch %d: rank %d exited with %d%s\n", epoch, rank, code,
                 signaled ? " (signal)" : "");
    if (code != 0 && res.rank < 0) {
      res.code = code;
      res.rank = rank;
      res.lost = signaled || code == kTempFail;
      kill_all(SIGTERM);                       // gang failure: stop the peers
      kill_deadline = time(nullptr) + o.grace;
      if (fork() == 0) {                       // escalate to SIGKILL after the grace period
        sleep((unsigned)o.grace);
        _exit(0);
      }
    }
    if (kill_deadline && time(nullptr) > kill_deadline) kill_all(SIGKILL);
  }
  return res;
}

int rm_entry(const char* path, const struct stat*, int, struct FTW*) {
  return remove(path) == 0 ? 0 : 0;
}

// Remove this launch's own checkpoint subdirectory (never the user's --checkpoint-dir itself):
// a new launch has a new subdirectory, so it never resumes a previous launch's stage outputs.
void remove_checkpoints(const Options& o) {
  if (o.ckpt_dir.empty()) return;
  struct stat st {};
  if (lstat(o.ckpt_dir.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) return;
  nftw(o.ckpt_dir.c_str(), rm_entry, 16, FTW_DEPTH | FTW_PHYS);
}

void log_event(const Options& o, const std::string& json) {
  std::fprintf(stderr, "[dryad-launch] %s\n", json.c_str());
  if (o.log_dir.empty()) return;
  const std::string path = o.log_dir + "/launcher.jsonl";
  if (FILE* f = std::fopen(path.c_str(), "a")) {
    std::fprintf(f, "%s\n", json.c_str());
    std::fclose(f);
  }
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
  int i = 1;
  for (; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--") { ++i; break; }
    if (a == "--gpus" && i + 1 < argc) o.n = std::atoi(argv[++i]);
    else if (a == "--master-port" && i + 1 < argc) o.port = std::atoi(argv[++i]);
    else if (a == "--log-dir" && i + 1 < argc) o.log_dir = argv[++i];
    else if (a == "--grace-seconds" && i + 1 < argc) o.grace = std::atoi(argv[++i]);
    else if (a == "--max-restarts" && i + 1 < argc) o.max_restarts = std::atoi(argv[++i]);
    else if (a == "--checkpoint-dir" && i + 1 < argc) o.ckpt_dir = argv[++i];
    else return usage();
  }
  if (i >= argc || o.n < 1 || o.n > 64 || o.max_restarts < 0) return usage();
  o.prog = argv + i;
  if (!o.log_dir.empty()) mkdir(o.log_dir.c_str(), 0755);
  if (o.ckpt_dir.empty() && o.max_restarts > 0) {
    // relaunches need the persisted stage outputs of the lost gang: by default they go to host
    // memory that outlives the rank processes (tmpfs), else next to the logs
    struct stat shm {};
    if (stat("/dev/shm", &shm) == 0 && S_ISDIR(shm.st_mode) && access("/dev/shm", W_OK) == 0) o.ckpt_dir = "/dev/shm";
    else if (!o.log_dir.empty()) o.ckpt_dir = o.log_dir;
  }
  if (!o.ckpt_dir.empty()) {
    struct stat st {};
    if (stat(o.ckpt_dir.c_str(), &st) != 0) {
      if (mkdir(o.ckpt_dir.c_str(), 0755) != 0) { std::perror("--checkpoint-dir"); return 2; }
    } else if (!S_ISDIR(st.st_mode)) {
      std::fprintf(stderr, "[dryad-launch] --checkpoint-dir %s is not a directory\n", o.ckpt_dir.c_str());
      return 2;
    }
    o.ckpt_dir += "/dryad-ckpt-" + std::to_string(getpid());
    remove_checkpoints(o);                     // a stale one of a recycled pid
    if (mkdir(o.ckpt_dir.c_str(), 0700) != 0) { std::perror("checkpoint subdirectory"); return 2; }
  }
  struct sigaction sa {};
  sa.sa_handler = on_signal;
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGTERM, &sa, nullptr);

  std::string reason;
  for (int epoch = 0;; ++epoch) {
    const GangResult r = run_gang(o, epoch, reason);
    if (r.rank < 0) {
      if (epoch > 0) log_event(o, "{\"ev\":\"job_complete\",\"epoch\":" + std::to_string(epoch) + "}");
      remove_checkpoints(o);
      return 0;
    }
    if (!r.lost || epoch >= o.max_restarts || r.rank >= o.n) {
      std::fprintf(stderr, "[dryad-launch] job failed: rank %d status %d\n", r.rank, r.code);
      remove_checkpoints(o);
      return r.code;
    }
    reason = "rank " + std::to_string(r.rank) + " lost (status " + std::to_string(r.code) + ")";
    log_event(o, "{\"ev\":\"gang_relaunch\",\"epoch\":" + std::to_string(epoch + 1) + ",\"rank\":" +
                     std::to_string(r.rank) + ",\"status\":" + std::to_string(r.code) + ",\"reason\":\"" + reason + "\"}");
  }
}
