// dryad-launch: start one worker process per GPU of the local node (reference A-7 job
// submission / H-3 ProcessService: LocalJobSubmission.cs starts the graph manager and a vertex
// host per computer; here every rank is a peer SPMD process over RCCL).
//
//   dryad-launch --gpus N [--master-port P] [--log-dir DIR] [--grace-seconds S] -- prog args...
//
// Each child gets RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
// MASTER_PORT (the torch.distributed env:// contract) and runs in its own process group.  The
// launcher waits for all ranks; the first rank that fails (non-zero exit or signal) makes it
// SIGTERM the others (SIGKILL after the grace period) so a dead rank never leaves the rest hung
// in a collective — the gang-failure rule of DrGang/DrCohort.  Exit status = first failure's.
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fcntl.h>
#include <string>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>
#include <vector>

namespace {

std::vector<pid_t> g_children;
volatile sig_atomic_t g_stop = 0;

void on_signal(int sig) {
  g_stop = sig;
}

void kill_all(int sig) {
  for (pid_t p : g_children)
    if (p > 0) kill(-p, sig);
}

int usage() {
  std::fprintf(stderr,
               "usage: dryad-launch --gpus N [--master-port P] [--log-dir DIR] [--grace-seconds S] -- prog args...\n");
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  int n = 1, port = 29511, grace = 10;
  std::string log_dir;
  int i = 1;
  for (; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--") { ++i; break; }
    if (a == "--gpus" && i + 1 < argc) n = std::atoi(argv[++i]);
    else if (a == "--master-port" && i + 1 < argc) port = std::atoi(argv[++i]);
    else if (a == "--log-dir" && i + 1 < argc) log_dir = argv[++i];
    else if (a == "--grace-seconds" && i + 1 < argc) grace = std::atoi(argv[++i]);
    else return usage();
  }
  if (i >= argc || n < 1 || n > 64) return usage();
  if (!log_dir.empty()) mkdir(log_dir.c_str(), 0755);
  struct sigaction sa {};
  sa.sa_handler = on_signal;
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGTERM, &sa, nullptr);

  for (int r = 0; r < n; ++r) {
    pid_t pid = fork();
    if (pid < 0) {
      std::perror("fork");
      kill_all(SIGTERM);
      return 1;
    }
    if (pid == 0) {
      setpgid(0, 0);
      const std::string rs = std::to_string(r), ns = std::to_string(n), ps = std::to_string(port);
      setenv("RANK", rs.c_str(), 1);
      setenv("LOCAL_RANK", rs.c_str(), 1);
      setenv("WORLD_SIZE", ns.c_str(), 1);
      setenv("LOCAL_WORLD_SIZE", ns.c_str(), 1);
      setenv("GROUP_RANK", "0", 1);
      setenv("MASTER_ADDR", "127.0.0.1", 1);
      setenv("MASTER_PORT", ps.c_str(), 1);
      if (!getenv("HSA_ENABLE_IPC_MODE_LEGACY")) setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0", 1);
      if (!log_dir.empty()) {
        const std::string path = log_dir + "/rank" + rs + ".log";
        int fd = open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0644);
        if (fd >= 0) {
          dup2(fd, 1);
          dup2(fd, 2);
          close(fd);
        }
      }
      execvp(argv[i], argv + i);
      std::perror("execvp");
      _exit(127);
    }
    setpgid(pid, pid);
    g_children.push_back(pid);
  }

  int first_fail = 0, first_rank = -1, alive = n;
  time_t kill_deadline = 0;
  while (alive > 0) {
    int status = 0;
    pid_t pid = waitpid(-1, &status, 0);
    if (pid < 0) {
      if (g_stop) {
        kill_all(SIGTERM);
        g_stop = 0;
        if (!kill_deadline) kill_deadline = time(nullptr) + grace;
        continue;
      }
      if (kill_deadline && time(nullptr) > kill_deadline) kill_all(SIGKILL);
      continue;
    }
    int rank = -1;
    for (int r = 0; r < n; ++r)
      if (g_children[r] == pid) rank = r;
    if (rank < 0) continue;
    g_children[rank] = -1;
    --alive;
    const int code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + WTERMSIG(status);
    std::fprintf(stderr, "[dryad-launch] rank %d exited with %d\n", rank, code);
    if (code != 0 && first_rank < 0) {
      first_fail = code;
      first_rank = rank;
      kill_all(SIGTERM);                       // gang failure: stop the peers
      kill_deadline = time(nullptr) + grace;
      if (fork() == 0) {                       // escalate to SIGKILL after the grace period
        sleep((unsigned)grace);
        _exit(0);
      }
    }
    if (kill_deadline && time(nullptr) > kill_deadline) kill_all(SIGKILL);
  }
  if (first_rank >= 0) std::fprintf(stderr, "[dryad-launch] job failed: rank %d status %d\n", first_rank, first_fail);
  return first_fail;
}
