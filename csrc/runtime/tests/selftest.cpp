// Native runtime self-test, built under AddressSanitizer+UBSan and ThreadSanitizer by
// tests/test_sanitizers.py ("build C++ with -fsanitize=address,undefined and TSAN
// targets for the scheduler/channel code").  Exercises the job graph state machine (failures,
// read-error upstream invalidation, speculative duplicates, gangs), the codec round trip, text
// splitting and the WorkQueue / async file reads under concurrency.
#include <atomic>
#include <cassert>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../codec.h"
#include "../jobgraph.h"
#include "../partreader.h"
#include "../pump.h"
#include "../workqueue.h"

using namespace dryad;

#define CHECK(c)                                                                  \
  do {                                                                            \
    if (!(c)) {                                                                   \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

static int test_jobgraph() {
  Params p;
  p.max_failures = 3;
  JobGraph g(p);
  const int s0 = g.add_stage("read", 4, true, false);
  const int s1 = g.add_stage("agg", 2, false, true);
  std::vector<int> a, b;
  for (int i = 0; i < 4; ++i) a.push_back(g.add_vertex(s0, i));
  for (int i = 0; i < 2; ++i) b.push_back(g.add_vertex(s1, i));
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 2; ++j) g.add_edge(a[i], j, b[j], i);
  g.start(0.0);
  double now = 0;
  int guard = 0;
  bool injected_fail = false, injected_read_error = false;
  while (!g.done() && !g.failed() && guard++ < 1000) {
    auto ready = g.take_ready(8, now);
    for (auto& it : ready) {
      g.on_running(it.vertex, it.version, 0, now);
      now += 0.5;
      if (!injected_fail && it.vertex == a[2]) {
        injected_fail = true;
        g.on_failed(it.vertex, it.version, now, -1, "injected");
        continue;
      }
      if (!injected_read_error && it.vertex == b[1]) {
        injected_read_error = true;
        g.on_failed(it.vertex, it.version, now, 3 * 2 + 1, "bad input");   // global edge a[3] -> b[1]
        continue;
      }
      bool accepted = false;
      g.on_completed(it.vertex, it.version, now, 10, 20, &accepted);
    }
    for (auto& d : g.check_duplicates(now)) (void)d;
    g.drain_events();
  }
  CHECK(g.done());
  CHECK(!g.failed());
  CHECK(g.completed_version(a[2]) >= 1);
  CHECK(g.completed_version(a[3]) >= 1);   // upstream of the read error was re-executed
  const std::string st = g.statistics_json();
  CHECK(st.find("\"stages\"") != std::string::npos);
  return 0;
}

static int test_codec() {
  std::vector<FieldKind> schema = {FieldKind::I32, FieldKind::String, FieldKind::F64, FieldKind::I64};
  const size_t n = 5000;
  std::vector<int32_t> c0(n);
  std::vector<double> c2(n);
  std::vector<int64_t> c3(n);
  StringColumn sc;
  sc.offsets.push_back(0);
  std::mt19937 rng(7);
  for (size_t i = 0; i < n; ++i) {
    c0[i] = (int32_t)rng();
    c2[i] = (double)i / 7.0;
    c3[i] = (int64_t)rng() << 20;
    std::string s(rng() % 300, 'a' + (char)(i % 26));
    if (i % 17 == 0) s += "\xc3\xa9\xe2\x82\xac";   // multi-byte UTF-8
    sc.data.insert(sc.data.end(), s.begin(), s.end());
    sc.offsets.push_back((int64_t)sc.data.size());
  }
  std::vector<const uint8_t*> fixed = {reinterpret_cast<const uint8_t*>(c0.data()), nullptr,
                                       reinterpret_cast<const uint8_t*>(c2.data()),
                                       reinterpret_cast<const uint8_t*>(c3.data())};
  std::vector<const StringColumn*> strs = {nullptr, &sc, nullptr, nullptr};
  auto bytes = encode_records(n, schema, fixed, strs);
  std::vector<std::vector<uint8_t>> outf;
  std::vector<StringColumn> outs;
  const size_t got = decode_records(bytes.data(), bytes.size(), schema, outf, outs);
  CHECK(got == n);
  CHECK(std::memcmp(outf[0].data(), c0.data(), n * 4) == 0);
  CHECK(std::memcmp(outf[3].data(), c3.data(), n * 8) == 0);
  CHECK(outs[1].data == sc.data && outs[1].offsets == sc.offsets);
  bool threw = false;   // truncated stream must throw, not read out of bounds
  try {
    decode_records(bytes.data(), bytes.size() - 3, schema, outf, outs);
  } catch (const std::runtime_error&) {
    threw = true;
  }
  CHECK(threw);
  std::vector<int64_t> st, en;
  const char* text = "a\r\nbb\rccc\n\nlast";
  split_lines(reinterpret_cast<const uint8_t*>(text), std::strlen(text), st, en);
  CHECK(st.size() == 5);
  return 0;
}

static int test_workqueue(const std::string& dir) {
  WorkQueue q(6);
  std::atomic<int> sum{0};
  for (int i = 0; i < 2000; ++i) q.submit([&sum, i] { sum += i; });
  q.drain();
  CHECK(sum.load() == 1999 * 2000 / 2);
  std::vector<std::string> paths;
  for (int i = 0; i < 16; ++i) {
    const std::string p = dir + "/f" + std::to_string(i);
    std::string data(1000 + i * 37, (char)('A' + i));
    write_file_atomic(p, reinterpret_cast<const uint8_t*>(data.data()), data.size());
    paths.push_back(p);
  }
  paths.push_back(dir + "/missing");
  auto b = read_files_async(q, paths);
  for (size_t i = 0; i < paths.size(); ++i) wait_read(*b, i);
  for (int i = 0; i < 16; ++i) CHECK(b->data[i].size() == (size_t)(1000 + i * 37) && b->data[i][0] == 'A' + i);
  CHECK(!b->errors[16].empty());
  // concurrent submitters
  std::vector<std::thread> ts;
  std::atomic<int> cnt{0};
  for (int t = 0; t < 4; ++t)
    ts.emplace_back([&] {
      for (int i = 0; i < 500; ++i) q.submit([&cnt] { cnt++; });
    });
  for (auto& t : ts) t.join();
  q.drain();
  CHECK(cnt.load() == 2000);
  return 0;
}

// the job manager pump under concurrent posters (run under TSan by tests/test_sanitizers.py)
static int test_pump() {
  dryad::MessagePump p;
  constexpr int kThreads = 4, kEach = 2000;
  std::vector<std::thread> th;
  for (int t = 0; t < kThreads; ++t)
    th.emplace_back([&p, t] {
      for (int i = 0; i < kEach; ++i) {
        if (i % 100 == 0) p.post_after(1, 2, t);
        p.post(1, (int64_t)t * kEach + i);
      }
    });
  int64_t got = 0, timers = 0, sum = 0;
  while (got < kThreads * kEach || timers < kThreads * (kEach / 100)) {
    for (auto& m : p.wait(-1)) {
      if (m.kind == 1) {
        ++got;
        sum += m.payload;
      } else {
        ++timers;
      }
    }
  }
  for (auto& x : th) x.join();
  const int64_t n = (int64_t)kThreads * kEach;
  CHECK(sum == n * (n - 1) / 2);
  CHECK(p.wait(0).empty());
  p.close();
  CHECK(p.wait(-1).empty());
  return 0;
}

// ChunkReader: buffers are (address, size) pairs; one smaller than a chunk is refused before any
// reader thread starts; a read through a ring smaller than the file returns every byte in order.
static int test_chunk_reader(const std::string& dir) {
  const std::string path = dir + "/chunkreader.bin";
  std::vector<uint8_t> data(1000003);
  for (size_t i = 0; i < data.size(); ++i) data[i] = (uint8_t)(i * 2654435761u >> 13);
  {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(data.data()), (std::streamsize)data.size());
  }
  const int64_t chunk = 65536;
  std::vector<std::vector<uint8_t>> ring(3, std::vector<uint8_t>(chunk));
  std::vector<uint8_t> small(chunk - 1);
  bool refused = false;
  try {
    ChunkReader bad(path, 0, -1, chunk, {{(uint64_t)ring[0].data(), chunk}, {(uint64_t)small.data(), chunk - 1}}, 2);
  } catch (const std::invalid_argument&) {
    refused = true;
  }
  CHECK(refused);
  refused = false;
  try {
    ChunkReader bad(path, 0, -1, chunk, {{0, chunk}}, 1);
  } catch (const std::invalid_argument&) {
    refused = true;
  }
  CHECK(refused);
  std::vector<std::pair<uint64_t, int64_t>> bufs;
  for (auto& b : ring) bufs.emplace_back((uint64_t)b.data(), (int64_t)b.size());
  ChunkReader rd(path, 17, -1, chunk, bufs, 3);
  CHECK(rd.size() == (int64_t)data.size() - 17);
  std::vector<uint8_t> got(rd.size());
  ReadyChunk c;
  int64_t seen = 0;
  while (rd.next(&c, -1)) {
    CHECK(c.slot >= 0 && c.bytes <= chunk);
    std::memcpy(got.data() + c.chunk * chunk, ring[c.slot].data(), (size_t)c.bytes);
    seen += c.bytes;
    rd.release(c.slot);
  }
  CHECK(rd.error().empty());
  CHECK(seen == rd.size());
  CHECK(std::memcmp(got.data(), data.data() + 17, got.size()) == 0);
  std::remove(path.c_str());
  return 0;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  if (int r = test_jobgraph()) return r;
  if (int r = test_codec()) return r;
  if (int r = test_workqueue(dir)) return r;
  if (int r = test_pump()) return r;
  if (int r = test_chunk_reader(dir)) return r;
  std::printf("SELFTEST_OK\n");
  return 0;
}
