// percall_bench.cpp -- latency of the per-call drop-in path (what EngineThreadCausalLog does
// per determinant and per BufferResponse) through the C-ABI, single-threaded and with
// several threads working on different logs at once (the task threads appending while
// Netty threads slice).  Prints one JSON line.
//
//   append          clg_append of one 9-byte Timestamp record            (appendDeterminant)
//   has_offset      clg_has_delta + clg_offset_from_epoch                  (hasDelta / getOffset)
//   get_delta_<n>   size probe + fetch into host memory of an n-byte delta (getDeltaForConsumer)
//
// Build: g++ -O2 -std=c++17 tools/percall_bench.cpp -Iinclude -Lclonos_amd -lclonos_engine
//        -Wl,-rpath,$PWD/clonos_amd -lpthread -o tools/percall_bench
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "clonos_engine.h"

using clk = std::chrono::steady_clock;

static void die(const char* what, int st) {
  fprintf(stderr, "%s failed: %d %s\n", what, st, clg_last_error());
  exit(1);
}
#define CK(x)                      \
  do {                             \
    int s_ = (x);                  \
    if (s_ != CLG_OK) die(#x, s_); \
  } while (0)

struct Pct {
  double p50, p99, mean;
};
static Pct pct(std::vector<double>& v) {
  std::sort(v.begin(), v.end());
  double s = 0;
  for (double x : v) s += x;
  return Pct{v[v.size() / 2], v[size_t(v.size() * 0.99)], s / v.size()};
}

// One worker: its own log; a mix of appends and slices like one task + one Netty channel.
static void worker(clg_engine* e, uint32_t log, int iters, size_t delta, std::vector<double>* t_app,
                   std::vector<double>* t_has, std::vector<double>* t_get, std::atomic<int>* go) {
  uint8_t rec[9] = {1, 0, 0, 1, 0x8b, 0, 0, 0, 0};
  std::vector<uint8_t> out(delta + 256);
  clg_channel_id ch{0xC0FFEE, log};
  while (!go->load()) std::this_thread::yield();
  const int per_delta = int(std::max<size_t>(1, delta / 9));
  for (int i = 0; i < iters; ++i) {
    for (int k = 0; k < per_delta; ++k) {
      auto a = clk::now();
      CK(clg_append(e, log, 1, rec, 9));
      if (k == 0) t_app->push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
    }
    auto b = clk::now();
    int32_t has = 0, ofe = 0;
    CK(clg_has_delta(e, log, ch, 1, &has));
    if (has) CK(clg_offset_from_epoch(e, log, ch, &ofe));
    auto c = clk::now();
    uint32_t n = 0;
    int st = clg_get_delta(e, log, ch, 1, nullptr, 0, CLG_MEM_HOST, &n);
    while (st == CLG_E_CAPACITY) {
      if (out.size() < n) out.resize(n + 256);
      st = clg_get_delta(e, log, ch, 1, out.data(), uint32_t(out.size()), CLG_MEM_HOST, &n);
    }
    if (st != CLG_OK) die("get_delta", st);
    auto d = clk::now();
    t_has->push_back(std::chrono::duration<double, std::micro>(c - b).count());
    t_get->push_back(std::chrono::duration<double, std::micro>(d - c).count());
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  clg_config cfg;
  clg_config_default(&cfg);
  cfg.pool_segments = 1 << 16;
  cfg.ifl_pool_segments = 16;
  clg_engine* e = nullptr;
  CK(clg_engine_create(&cfg, &e));
  std::string json = "{\"metric\": \"per-call C-ABI latency (us)\", \"iters\": " + std::to_string(iters) + ", \"cases\": [";
  bool first = true;
  for (size_t delta : {16, 1024, 16384}) {
    for (int threads : {1, 8}) {
      std::vector<uint32_t> logs(threads);
      for (int t = 0; t < threads; ++t) {
        clg_causal_log_id id{};
        id.vertex_id = int16_t(1000 + t + 16 * int(delta % 7));
        id.is_main = 1;
        CK(clg_log_open(e, 0, &id, &logs[t]));
      }
      std::vector<std::vector<double>> ta(threads), th(threads), tg(threads);
      std::atomic<int> go{0};
      std::vector<std::thread> ws;
      auto t0 = clk::now();
      for (int t = 0; t < threads; ++t)
        ws.emplace_back(worker, e, logs[t], iters, delta, &ta[t], &th[t], &tg[t], &go);
      go = 1;
      for (auto& w : ws) w.join();
      const double wall = std::chrono::duration<double>(clk::now() - t0).count();
      std::vector<double> a, h, g;
      for (int t = 0; t < threads; ++t) {
        a.insert(a.end(), ta[t].begin(), ta[t].end());
        h.insert(h.end(), th[t].begin(), th[t].end());
        g.insert(g.end(), tg[t].begin(), tg[t].end());
      }
      const Pct pa = pct(a), ph = pct(h), pg = pct(g);
      char buf[768];
      snprintf(buf, sizeof buf,
               "%s{\"delta_bytes\": %zu, \"threads\": %d, \"append\": {\"p50\": %.2f, \"p99\": %.2f}, "
               "\"has_offset\": {\"p50\": %.2f, \"p99\": %.2f}, \"get_delta\": {\"p50\": %.2f, \"p99\": %.2f, "
               "\"mean\": %.2f}, \"slices_per_s\": %.0f}",
               first ? "" : ", ", delta, threads, pa.p50, pa.p99, ph.p50, ph.p99, pg.p50, pg.p99, pg.mean,
               double(threads) * iters / wall);
      json += buf;
      first = false;
      for (uint32_t l : logs) CK(clg_log_close(e, l));
    }
  }
  json += "]}";
  printf("%s\n", json.c_str());
  clg_engine_destroy(e);
  return 0;
}
