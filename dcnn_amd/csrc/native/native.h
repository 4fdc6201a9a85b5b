// Host-side C++ runtime of dcnn_amd (no GPU code): env loader, hardware info, thread
// affinity, message serialisation + TCP control plane, dataset parsers, augmentation.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace dcnn_native {

// env.cpp
std::map<std::string, std::string> parse_env_text(const std::string& text);
int load_env_file(const std::string& path, bool overwrite);

// hwinfo.cpp
struct CpuInfo {
  std::string vendor, model_name;
  int logical_cores = 0, physical_cores = 0, sockets = 0;
  double base_mhz = 0, max_mhz = 0;
  std::vector<std::string> flags;
  std::map<std::string, long> caches_kb;  // L1d/L1i/L2/L3
  long total_mem_kb = 0, avail_mem_kb = 0;
  long cgroup_mem_limit_bytes = -1;
  double cgroup_cpu_quota = -1;  // cores
  std::vector<int> pcores, ecores;
};
CpuInfo read_cpu_info();
std::vector<double> cpu_utilization(int sample_ms);  // per-core %, from /proc/stat deltas
double cpu_utilization_total(int sample_ms);
long process_rss_kb();
std::vector<std::pair<std::string, double>> thermal_zones();

// jpeg.cpp — baseline Huffman JPEG -> interleaved RGB8
bool decode_jpeg(const unsigned char* data, size_t n, std::vector<unsigned char>& rgb, int& w, int& h,
                 std::string* err);

// affinity (hwinfo.cpp)
int set_thread_affinity(const std::vector<int>& cpus);
std::vector<int> get_thread_affinity();

}  // namespace dcnn_native
