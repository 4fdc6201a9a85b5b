// .env loader (reference include/utils/env.hpp:41-137): KEY=VALUE lines, optional `export `,
// single/double quotes, `#` comments (full-line and trailing after whitespace), setenv.
#include "native.h"

#include <cstdlib>
#include <fstream>
#include <sstream>

namespace dcnn_native {

static std::string trim(const std::string& s) {
  size_t b = s.find_first_not_of(" \t\r\n");
  if (b == std::string::npos) return "";
  size_t e = s.find_last_not_of(" \t\r\n");
  return s.substr(b, e - b + 1);
}

std::map<std::string, std::string> parse_env_text(const std::string& text) {
  std::map<std::string, std::string> out;
  std::istringstream in(text);
  std::string line;
  while (std::getline(in, line)) {
    line = trim(line);
    if (line.empty() || line[0] == '#') continue;
    if (line.rfind("export ", 0) == 0) line = trim(line.substr(7));
    const size_t eq = line.find('=');
    if (eq == std::string::npos) continue;
    std::string key = trim(line.substr(0, eq));
    std::string val = trim(line.substr(eq + 1));
    if (key.empty()) continue;
    if (val.size() >= 2 && (val[0] == '"' || val[0] == '\'') && val.back() == val[0]) {
      val = val.substr(1, val.size() - 2);
    } else {
      // strip trailing comment " # ..."
      size_t h = val.find(" #");
      if (h == std::string::npos) h = val.find("\t#");
      if (h != std::string::npos) val = trim(val.substr(0, h));
    }
    out[key] = val;
  }
  return out;
}

int load_env_file(const std::string& path, bool overwrite) {
  std::ifstream f(path);
  if (!f.is_open()) return -1;
  std::stringstream ss;
  ss << f.rdbuf();
  int n = 0;
  for (const auto& kv : parse_env_text(ss.str())) {
    if (::setenv(kv.first.c_str(), kv.second.c_str(), overwrite ? 1 : 0) == 0) ++n;
  }
  return n;
}

}  // namespace dcnn_native
