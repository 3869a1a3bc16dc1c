// Native OpenB CSV readers -> SoA columns (the engines' input layout).
//
// Same parsing rules as the reference TraceParser (benchmarks/parser.py:9-122)
// and core/traces.py: header-addressed columns, an empty gpu_milli reads as 0,
// duration = deletion_time - creation_time, a missing required column is a
// KeyError (the multigpu*.csv traces have no gpu_spec / time columns), node
// rows keep dict semantics (a repeated `sn` keeps its first position and takes
// the last row's values).
#pragma once

#include <cstdint>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace fks {

struct MissingColumn : std::runtime_error {
  explicit MissingColumn(const std::string& c) : std::runtime_error(c) {}
};

// Minimal RFC-4180 line splitter (quotes, doubled quotes; no embedded newlines).
inline void split_csv_line(const std::string& line, std::vector<std::string>& out) {
  out.clear();
  std::string cur;
  bool q = false;
  for (size_t i = 0; i < line.size(); ++i) {
    const char c = line[i];
    if (q) {
      if (c == '"') {
        if (i + 1 < line.size() && line[i + 1] == '"') { cur.push_back('"'); ++i; }
        else q = false;
      } else {
        cur.push_back(c);
      }
    } else if (c == '"') {
      q = true;
    } else if (c == ',') {
      out.push_back(cur);
      cur.clear();
    } else if (c != '\r') {
      cur.push_back(c);
    }
  }
  out.push_back(cur);
}

struct CsvTable {
  std::vector<std::string> header;
  std::vector<std::vector<std::string>> rows;
  int col(const std::string& name) const {
    for (size_t i = 0; i < header.size(); ++i)
      if (header[i] == name) return (int)i;
    throw MissingColumn(name);
  }
};

inline CsvTable read_csv(const std::string& path) {
  std::ifstream in(path);
  if (!in) throw std::runtime_error("cannot open " + path);
  CsvTable t;
  std::string line;
  if (!std::getline(in, line)) return t;
  if (line.size() >= 3 && (unsigned char)line[0] == 0xEF) line = line.substr(3);   // UTF-8 BOM
  split_csv_line(line, t.header);
  std::vector<std::string> f;
  while (std::getline(in, line)) {
    if (line.empty() || line == "\r") continue;
    split_csv_line(line, f);
    f.resize(t.header.size());
    t.rows.push_back(f);
  }
  return t;
}

inline int64_t to_i64(const std::string& s, const char* what) {
  if (s.empty()) throw std::invalid_argument(std::string("empty ") + what);
  char* end = nullptr;
  const long long v = std::strtoll(s.c_str(), &end, 10);
  if (end == s.c_str() || *end != '\0') throw std::invalid_argument(std::string("bad integer in ") + what + ": " + s);
  return (int64_t)v;
}

struct PodColumns {
  std::vector<std::string> name, gpu_spec;
  std::vector<int64_t> cpu, mem, ctime, dur;
  std::vector<int32_t> ngpu, gmilli;
};

inline PodColumns load_pods(const std::string& path) {
  const CsvTable t = read_csv(path);
  const int c_name = t.col("name"), c_cpu = t.col("cpu_milli"), c_mem = t.col("memory_mib");
  const int c_ng = t.col("num_gpu"), c_gm = t.col("gpu_milli"), c_spec = t.col("gpu_spec");
  const int c_ct = t.col("creation_time"), c_dt = t.col("deletion_time");
  PodColumns p;
  const size_t n = t.rows.size();
  p.name.reserve(n); p.gpu_spec.reserve(n);
  for (const auto& r : t.rows) {
    p.name.push_back(r[c_name]);
    p.cpu.push_back(to_i64(r[c_cpu], "cpu_milli"));
    p.mem.push_back(to_i64(r[c_mem], "memory_mib"));
    p.ngpu.push_back((int32_t)to_i64(r[c_ng], "num_gpu"));
    p.gmilli.push_back(r[c_gm].empty() ? 0 : (int32_t)to_i64(r[c_gm], "gpu_milli"));
    p.gpu_spec.push_back(r[c_spec]);
    const int64_t ct = to_i64(r[c_ct], "creation_time");
    p.ctime.push_back(ct);
    p.dur.push_back(to_i64(r[c_dt], "deletion_time") - ct);
  }
  return p;
}

struct NodeColumns {
  std::vector<std::string> sn;
  std::vector<int64_t> cpu, mem;
  std::vector<int32_t> gpu_count, ngpus;       // CSV count / materialised GPU cards
  std::vector<int64_t> gpu_mem;                // per node: card memory (0 when no cards)
};

inline NodeColumns load_nodes(const std::string& path, const std::unordered_map<std::string, int64_t>& mem_map) {
  const CsvTable t = read_csv(path);
  const int c_sn = t.col("sn"), c_cpu = t.col("cpu_milli"), c_mem = t.col("memory_mib");
  const int c_gpu = t.col("gpu"), c_model = t.col("model");
  NodeColumns nc;
  std::unordered_map<std::string, size_t> pos;
  for (const auto& r : t.rows) {
    const std::string& sn = r[c_sn];
    const int32_t count = (int32_t)to_i64(r[c_gpu], "gpu");
    const auto it = mem_map.find(r[c_model]);
    const bool cards = count > 0 && it != mem_map.end();
    const int64_t cpu = to_i64(r[c_cpu], "cpu_milli"), mem = to_i64(r[c_mem], "memory_mib");
    auto p = pos.find(sn);
    size_t i;
    if (p == pos.end()) {
      i = nc.sn.size();
      pos.emplace(sn, i);
      nc.sn.push_back(sn);
      nc.cpu.push_back(0); nc.mem.push_back(0); nc.gpu_count.push_back(0); nc.ngpus.push_back(0);
      nc.gpu_mem.push_back(0);
    } else {
      i = p->second;   // dict semantics: first position, last values
    }
    nc.cpu[i] = cpu;
    nc.mem[i] = mem;
    nc.gpu_count[i] = count;
    nc.ngpus[i] = cards ? count : 0;
    nc.gpu_mem[i] = cards ? it->second : 0;
  }
  return nc;
}

}  // namespace fks
