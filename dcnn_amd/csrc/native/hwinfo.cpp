// Hardware info (reference src/utils/hardware_info.cpp: /proc/cpuinfo, /proc/meminfo,
// /proc/stat utilisation, cgroup limits, thermal zones, P/E-core topology) and thread
// affinity (src/utils/thread_affinity.cpp:175-194). GPU topology (MI355X, xGMI) is queried on
// the Python side through torch / rocm-smi; this file is host-only.
#include <pthread.h>
#include <sched.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <dirent.h>
#include <fstream>
#include <set>
#include <sstream>
#include <thread>

#include "native.h"

namespace dcnn_native {

static std::string read_file(const std::string& p) {
  std::ifstream f(p);
  if (!f.is_open()) return "";
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

static std::string trimw(const std::string& s) {
  size_t b = s.find_first_not_of(" \t\r\n");
  if (b == std::string::npos) return "";
  return s.substr(b, s.find_last_not_of(" \t\r\n") - b + 1);
}

CpuInfo read_cpu_info() {
  CpuInfo ci;
  std::istringstream in(read_file("/proc/cpuinfo"));
  std::string line;
  std::set<std::pair<int, int>> cores;
  std::set<int> sockets;
  int phys = -1, core = -1;
  double mhz_sum = 0;
  int mhz_n = 0;
  while (std::getline(in, line)) {
    const size_t c = line.find(':');
    if (c == std::string::npos) {
      if (phys >= 0 || core >= 0) cores.insert({phys, core});
      phys = core = -1;
      continue;
    }
    std::string k = trimw(line.substr(0, c)), v = trimw(line.substr(c + 1));
    if (k == "processor") ci.logical_cores++;
    else if (k == "vendor_id" && ci.vendor.empty()) ci.vendor = v;
    else if (k == "model name" && ci.model_name.empty()) ci.model_name = v;
    else if (k == "physical id") { phys = std::atoi(v.c_str()); sockets.insert(phys); }
    else if (k == "core id") core = std::atoi(v.c_str());
    else if (k == "cpu MHz") { mhz_sum += std::atof(v.c_str()); ++mhz_n; }
    else if (k == "flags" && ci.flags.empty()) {
      std::istringstream fs(v);
      std::string fl;
      while (fs >> fl) ci.flags.push_back(fl);
    }
  }
  if (phys >= 0 || core >= 0) cores.insert({phys, core});
  ci.physical_cores = cores.empty() ? ci.logical_cores : (int)cores.size();
  ci.sockets = sockets.empty() ? 1 : (int)sockets.size();
  ci.base_mhz = mhz_n ? mhz_sum / mhz_n : 0;
  const std::string mx = read_file("/sys/devices/system/cpu/cpu0/cpufreq/cpuinfo_max_freq");
  if (!mx.empty()) ci.max_mhz = std::atof(mx.c_str()) / 1000.0;
  // caches
  for (int i = 0; i < 8; ++i) {
    const std::string base = "/sys/devices/system/cpu/cpu0/cache/index" + std::to_string(i) + "/";
    const std::string lvl = trimw(read_file(base + "level"));
    if (lvl.empty()) break;
    const std::string type = trimw(read_file(base + "type"));
    const std::string sz = trimw(read_file(base + "size"));
    std::string name = "L" + lvl + (type == "Data" ? "d" : type == "Instruction" ? "i" : "");
    ci.caches_kb[name] = std::atol(sz.c_str());
  }
  // memory
  std::istringstream mi(read_file("/proc/meminfo"));
  while (std::getline(mi, line)) {
    long v = 0;
    char key[64];
    if (std::sscanf(line.c_str(), "%63[^:]: %ld", key, &v) == 2) {
      if (std::string(key) == "MemTotal") ci.total_mem_kb = v;
      if (std::string(key) == "MemAvailable") ci.avail_mem_kb = v;
    }
  }
  // cgroup v2 / v1 limits (containers)
  std::string lim = trimw(read_file("/sys/fs/cgroup/memory.max"));
  if (lim.empty()) lim = trimw(read_file("/sys/fs/cgroup/memory/memory.limit_in_bytes"));
  if (!lim.empty() && lim != "max") ci.cgroup_mem_limit_bytes = std::atol(lim.c_str());
  std::string cpu = trimw(read_file("/sys/fs/cgroup/cpu.max"));
  if (!cpu.empty()) {
    std::istringstream cs(cpu);
    std::string q, p;
    cs >> q >> p;
    if (q != "max" && !p.empty()) ci.cgroup_cpu_quota = std::atof(q.c_str()) / std::atof(p.c_str());
  }
  // hybrid topology: cores whose max frequency is the highest are P-cores
  std::map<int, long> maxf;
  for (int c = 0; c < ci.logical_cores; ++c) {
    const std::string f = trimw(read_file("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/cpufreq/cpuinfo_max_freq"));
    maxf[c] = f.empty() ? 0 : std::atol(f.c_str());
  }
  long top = 0;
  for (auto& kv : maxf) top = std::max(top, kv.second);
  for (auto& kv : maxf) {
    if (top == 0 || kv.second >= top * 0.9) ci.pcores.push_back(kv.first);
    else ci.ecores.push_back(kv.first);
  }
  return ci;
}

struct StatSample { std::vector<unsigned long long> busy, total; };

static StatSample read_stat() {
  StatSample s;
  std::istringstream in(read_file("/proc/stat"));
  std::string line;
  while (std::getline(in, line)) {
    if (line.rfind("cpu", 0) != 0) break;
    std::istringstream ls(line);
    std::string name;
    ls >> name;
    unsigned long long v, tot = 0, idle = 0;
    int i = 0;
    while (ls >> v) {
      tot += v;
      if (i == 3 || i == 4) idle += v;  // idle + iowait
      ++i;
    }
    s.busy.push_back(tot - idle);
    s.total.push_back(tot);
  }
  return s;
}

std::vector<double> cpu_utilization(int sample_ms) {
  StatSample a = read_stat();
  std::this_thread::sleep_for(std::chrono::milliseconds(sample_ms));
  StatSample b = read_stat();
  std::vector<double> out;
  for (size_t i = 1; i < a.total.size() && i < b.total.size(); ++i) {
    const double dt = (double)(b.total[i] - a.total[i]);
    out.push_back(dt > 0 ? 100.0 * (double)(b.busy[i] - a.busy[i]) / dt : 0.0);
  }
  return out;
}

double cpu_utilization_total(int sample_ms) {
  StatSample a = read_stat();
  std::this_thread::sleep_for(std::chrono::milliseconds(sample_ms));
  StatSample b = read_stat();
  if (a.total.empty() || b.total.empty()) return 0;
  const double dt = (double)(b.total[0] - a.total[0]);
  return dt > 0 ? 100.0 * (double)(b.busy[0] - a.busy[0]) / dt : 0.0;
}

long process_rss_kb() {
  std::istringstream in(read_file("/proc/self/status"));
  std::string line;
  while (std::getline(in, line)) {
    long v;
    if (std::sscanf(line.c_str(), "VmRSS: %ld", &v) == 1) return v;
  }
  return -1;
}

std::vector<std::pair<std::string, double>> thermal_zones() {
  std::vector<std::pair<std::string, double>> out;
  for (int i = 0; i < 64; ++i) {
    const std::string base = "/sys/class/thermal/thermal_zone" + std::to_string(i) + "/";
    const std::string t = trimw(read_file(base + "temp"));
    if (t.empty()) break;
    out.push_back({trimw(read_file(base + "type")), std::atof(t.c_str()) / 1000.0});
  }
  return out;
}

int set_thread_affinity(const std::vector<int>& cpus) {
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus) CPU_SET(c, &set);
  return pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

std::vector<int> get_thread_affinity() {
  cpu_set_t set;
  CPU_ZERO(&set);
  std::vector<int> out;
  if (pthread_getaffinity_np(pthread_self(), sizeof(set), &set) != 0) return out;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &set)) out.push_back(c);
  return out;
}

}  // namespace dcnn_native
