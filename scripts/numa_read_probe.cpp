// Host DRAM read bandwidth under N concurrent readers (can one host feed
// 8 x 56 GB/s of pinned-buffer H2D reads?). Each reader process binds to the allowed CPUs of one
// NUMA node, first-touches its own buffer there, and streams it with T threads (read-only sum),
// reporting GB/s on stdout as one JSON line. Launched by scripts/numa_read_probe.py.
//
//   numa_read_probe <node> <threads> <MiB> <seconds>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

static std::vector<int> node_cpus(int node) {
  std::vector<int> out;
  std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string s;
  if (!std::getline(f, s)) return out;
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  sched_getaffinity(0, sizeof(allowed), &allowed);
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    std::string r = s.substr(i, j - i);
    size_t d = r.find('-');
    int a = atoi(r.c_str()), b = d == std::string::npos ? a : atoi(r.c_str() + d + 1);
    for (int c = a; c <= b; ++c)
      if (CPU_ISSET(c, &allowed)) out.push_back(c);
    i = j + 1;
  }
  return out;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s node threads MiB seconds\n", argv[0]);
    return 2;
  }
  const int node = atoi(argv[1]), T = atoi(argv[2]);
  const size_t bytes = (size_t)atoll(argv[3]) << 20;
  const double secs = atof(argv[4]);
  std::vector<int> cpus = node_cpus(node);
  if (!cpus.empty()) {
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int c : cpus) CPU_SET(c, &set);
    sched_setaffinity(0, sizeof(set), &set);
  }
  const size_t n = bytes / 8;
  uint64_t* buf = static_cast<uint64_t*>(aligned_alloc(4096, n * 8));
  if (!buf) return 3;
  std::vector<std::thread> th;
  const size_t per = n / T;
  for (int t = 0; t < T; ++t)  // first touch by the reading threads (local pages)
    th.emplace_back([=] { memset(buf + t * per, 1, per * 8); });
  for (auto& x : th) x.join();
  th.clear();
  std::atomic<uint64_t> total{0};
  std::atomic<uint64_t> sink{0};
  const auto t0 = std::chrono::steady_clock::now();
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      uint64_t acc = 0, done = 0;
      const uint64_t* p = buf + t * per;
      while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
        uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
        for (size_t i = 0; i + 4 <= per; i += 4) {
          a0 += p[i];
          a1 += p[i + 1];
          a2 += p[i + 2];
          a3 += p[i + 3];
        }
        acc += a0 ^ a1 ^ a2 ^ a3;
        done += per * 8;
      }
      total += done;
      sink += acc;
    });
  for (auto& x : th) x.join();
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("{\"node\": %d, \"cpus\": %zu, \"threads\": %d, \"gbps\": %.2f, \"chk\": %llu}\n", node, cpus.size(), T,
         total.load() / dt / 1e9, (unsigned long long)(sink.load() & 1));
  free(buf);
  return 0;
}
