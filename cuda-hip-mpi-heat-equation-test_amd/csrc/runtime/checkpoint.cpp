// Checkpoint / restart for the native CLI, in the SAME on-disk format as the
// Python driver (utils/checkpoint.py, "heat2d-checkpoint-v2", ckpt.hpp):
//   DIR/step-NNNNNNNNNNNN/rankNNNNN.npy  each rank's owned rows (NumPy v1 header, C order)
//   DIR/step-NNNNNNNNNNNN/meta.json      problem + solver parameters + completed step count
//   DIR/latest                           the newest complete step (atomic commit point)
// so a run can checkpoint from `heat2d --gpus 8` and resume under torchrun
// (or the other way round), on any rank count: restart reads each writer
// file's row range that overlaps this rank's slab. The reference has no
// restart at all (its int.dat / soln*.dat dumps are never read back;
// SURVEY.md §5).
#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <vector>

#include "heat2d/capi.h"
#include "heat2d/ckpt.hpp"
#include "heat2d/runtime.hpp"

namespace heat2d {
namespace ckpt {

namespace {

constexpr const char* kFormat = "heat2d-checkpoint-v2";
constexpr const char* kFormatV1 = "heat2d-checkpoint-v1";  // flat layout, still readable

std::string join(const std::string& dir, const std::string& name) { return dir + "/" + name; }

std::string step_name(int64_t step) {
  char b[32];
  std::snprintf(b, sizeof(b), "step-%012lld", (long long)step);
  return b;
}

bool exists(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0;
}

// data of `path` (a file or a directory: its entries) on stable storage
void fsync_path(const std::string& path) {
  const int fd = ::open(path.c_str(), O_RDONLY);
  HEAT2D_REQUIRE(fd >= 0, "cannot open " + path + " to fsync");
  const int rc = ::fsync(fd);
  const int err = errno;  // (close may overwrite it)
  ::close(fd);
  HEAT2D_REQUIRE(rc == 0 || err == EINVAL, "fsync failed on " + path);
}

std::string parent_dir(const std::string& path) {
  const size_t p = path.find_last_of('/');
  return p == std::string::npos ? "." : (p == 0 ? "/" : path.substr(0, p));
}

void write_atomic(const std::string& path, const std::string& text) {
  const std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  HEAT2D_REQUIRE(f != nullptr, "cannot write " + tmp);
  const bool ok = std::fwrite(text.data(), 1, text.size(), f) == text.size() && std::fflush(f) == 0 &&
                  ::fsync(fileno(f)) == 0;
  HEAT2D_REQUIRE(std::fclose(f) == 0 && ok, "error writing " + tmp);
  HEAT2D_REQUIRE(std::rename(tmp.c_str(), path.c_str()) == 0, "cannot publish " + path);
  fsync_path(parent_dir(path));  // the rename itself
}

std::string rank_file(const std::string& dir, int rank) {
  char b[32];
  std::snprintf(b, sizeof(b), "rank%05d.npy", rank);
  return join(dir, b);
}

// closes on every exit path (the REQUIREs below throw)
struct File {
  FILE* f;
  File(const std::string& path, const char* mode) : f(std::fopen(path.c_str(), mode)) {
    HEAT2D_REQUIRE(f != nullptr, "cannot open " + path);
  }
  ~File() {
    if (f) std::fclose(f);
  }
  File(const File&) = delete;
  File& operator=(const File&) = delete;
};

std::string read_text(const std::string& path) {
  File f(path, "rb");
  std::string s;
  char buf[4096];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f.f)) > 0) s.append(buf, n);
  return s;
}

// Value of "key" in a flat JSON object (numbers or strings; enough for the
// meta.json both writers produce).
std::string json_value(const std::string& js, const std::string& key) {
  const std::string pat = "\"" + key + "\"";
  size_t p = js.find(pat);
  HEAT2D_REQUIRE(p != std::string::npos, "checkpoint meta.json lacks \"" + key + "\"");
  p = js.find(':', p + pat.size());
  HEAT2D_REQUIRE(p != std::string::npos, "malformed meta.json");
  ++p;
  while (p < js.size() && (js[p] == ' ' || js[p] == '\n' || js[p] == '\t' || js[p] == '\r')) ++p;
  HEAT2D_REQUIRE(p < js.size(), "malformed meta.json");
  if (js[p] == '"') {
    const size_t q = js.find('"', p + 1);
    HEAT2D_REQUIRE(q != std::string::npos, "malformed meta.json string");
    return js.substr(p + 1, q - p - 1);
  }
  size_t q = p;
  while (q < js.size() && js[q] != ',' && js[q] != '}' && js[q] != '\n') ++q;
  return js.substr(p, q - p);
}

struct NpyInfo {
  int64_t rows = 0, cols = 0;
  int dtype = 1;       // 0 fp32, 1 fp64
  long data_off = 0;   // byte offset of the array data
};

NpyInfo npy_header(FILE* f, const std::string& path) {
  unsigned char head[10];
  HEAT2D_REQUIRE(std::fread(head, 1, 10, f) == 10 && std::memcmp(head, "\x93NUMPY", 6) == 0,
                 path + ": not a .npy file");
  const int major = head[6];
  size_t hlen = 0;
  long off = 0;
  if (major == 1) {
    hlen = (size_t)head[8] | ((size_t)head[9] << 8);
    off = 10;
  } else {
    unsigned char ext[2];
    HEAT2D_REQUIRE(std::fread(ext, 1, 2, f) == 2, path + ": truncated header");
    hlen = (size_t)head[8] | ((size_t)head[9] << 8) | ((size_t)ext[0] << 16) | ((size_t)ext[1] << 24);
    off = 12;
  }
  HEAT2D_REQUIRE(hlen > 0 && hlen < (1u << 20), path + ": bad header length");
  std::string h(hlen, '\0');
  HEAT2D_REQUIRE(std::fread(&h[0], 1, hlen, f) == hlen, path + ": truncated header");
  NpyInfo info;
  info.data_off = off + (long)hlen;
  if (h.find("'<f8'") != std::string::npos) info.dtype = 1;
  else if (h.find("'<f4'") != std::string::npos) info.dtype = 0;
  else fail(__FILE__, __LINE__, path + ": dtype is not little-endian f4/f8");
  HEAT2D_REQUIRE(h.find("'fortran_order': False") != std::string::npos, path + ": Fortran-ordered array");
  const size_t sp = h.find("'shape':");
  HEAT2D_REQUIRE(sp != std::string::npos, path + ": no shape");
  long long r = 0, c = 0;
  HEAT2D_REQUIRE(std::sscanf(h.c_str() + sp, "'shape': (%lld, %lld)", &r, &c) == 2 && r >= 0 && c > 0,
                 path + ": expected a 2-D shape");
  info.rows = r;
  info.cols = c;
  return info;
}

}  // namespace

// (step, generation) of a step directory name "step-<12 digits>[-<digits>]"
// (generation 0: the bare name; any all-digit suffix counts, the legacy -N
// too); false for anything else. Pruning orders saves by this key, not by
// name: a legacy step-X-7 and a new step-X-000008 compare by their numbers.
static bool step_key(const std::string& n, long long* step, long long* gen) {
  if (n.compare(0, 5, "step-") != 0 || n.size() < 5 + 12) return false;
  for (size_t i = 5; i < 17; ++i)
    if (!std::isdigit((unsigned char)n[i])) return false;
  *step = std::atoll(n.c_str() + 5);
  *gen = 0;
  if (n.size() == 17) return true;
  if (n[17] != '-' || n.size() == 18) return false;
  for (size_t i = 18; i < n.size(); ++i)
    if (!std::isdigit((unsigned char)n[i])) return false;
  *gen = std::atoll(n.c_str() + 18);
  return true;
}

// A name no earlier save of this step used, ordered after all of them (and
// before the next step) by step_key: `base` for the first save, then
// base-000001, base-000002, ... one past the highest generation present
// (legacy -N suffixes included) — never a gap a pruned generation left.
std::string step_dir_name(const std::string& dir, int64_t step) {
  const std::string base = step_name(step);
  bool any = false;
  long long gmax = 0;
  if (DIR* d = ::opendir(dir.c_str())) {
    while (dirent* e = ::readdir(d)) {
      long long st = 0, g = 0;
      if (!step_key(e->d_name, &st, &g) || st != (long long)step) continue;
      any = true;
      gmax = std::max(gmax, g);
    }
    ::closedir(d);
  }
  if (!any) return base;
  char b[16];
  std::snprintf(b, sizeof(b), "-%06lld", gmax + 1);
  return base + b;
}

void write_rank(const std::string& dir, const std::string& name, int rank, Solver& s) {
  ::mkdir(dir.c_str(), 0755);  // all ranks may race on it: EEXIST is fine
  const std::string sd = join(dir, name);
  ::mkdir(sd.c_str(), 0755);
  const SlabLayout& L = s.layout();
  std::vector<char> host((size_t)(L.nrows * L.ncols) * dtype_size(s.dtype()));
  s.download(host.data(), L.ncols);
  const std::string path = rank_file(sd, rank);
  if (heat2d_write_npy(path.c_str(), (int)s.dtype(), host.data(), L.nrows, L.ncols, L.ncols))
    fail(__FILE__, __LINE__, heat2d_last_error());
  fsync_path(path);
}

void write_meta(const std::string& dir, const std::string& name, const Meta& m) {
  char buf[1024];
  std::snprintf(buf, sizeof(buf),
                "{\n \"format\": \"%s\",\n \"step\": %lld,\n \"nranks\": %d,\n \"dtype\": \"%s\",\n"
                " \"n_owned\": %lld,\n \"n_input\": %lld,\n \"convention\": \"%s\",\n \"sigma\": %.17g,\n"
                " \"nu\": %.17g,\n \"dom_len\": %.17g,\n \"r\": %.17g,\n \"edge_shift\": %lld,\n"
                " \"writer\": \"heat2d-cli\"\n}\n",
                kFormat, (long long)m.step, m.nranks, m.dtype == 0 ? "fp32" : "fp64", (long long)m.n_owned,
                (long long)m.n_input, m.convention.c_str(), m.sigma, m.nu, m.dom_len, m.r, (long long)m.edge_shift);
  write_atomic(join(join(dir, name), "meta.json"), buf);  // + fsync of the step directory (rank files' entries)
  write_atomic(join(dir, "latest"), name + "\n");  // the commit point
  // prune: keep the two newest complete saves, ordered by (step, generation)
  std::vector<std::string> steps;
  if (DIR* d = ::opendir(dir.c_str())) {
    long long st = 0, g = 0;
    while (dirent* e = ::readdir(d))
      if (step_key(e->d_name, &st, &g)) steps.push_back(e->d_name);
    ::closedir(d);
  }
  std::sort(steps.begin(), steps.end(), [](const std::string& a, const std::string& b) {
    long long sa = 0, ga = 0, sb = 0, gb = 0;
    step_key(a, &sa, &ga);
    step_key(b, &sb, &gb);
    return sa != sb ? sa < sb : ga < gb;
  });
  const auto cur = std::find(steps.begin(), steps.end(), name);
  for (auto it = steps.begin(); cur != steps.end() && it + 1 < cur; ++it) {
    const std::string sd = join(dir, *it);
    if (DIR* d = ::opendir(sd.c_str())) {
      while (dirent* e = ::readdir(d))
        if (e->d_name[0] != '.') ::unlink(join(sd, e->d_name).c_str());
      ::closedir(d);
    }
    ::rmdir(sd.c_str());
  }
}

Meta read_meta(const std::string& dir) {
  std::string sd = dir;
  if (exists(join(dir, "latest"))) {
    std::string name = read_text(join(dir, "latest"));
    while (!name.empty() && (name.back() == '\n' || name.back() == ' ')) name.pop_back();
    sd = join(dir, name);
  }
  HEAT2D_REQUIRE(exists(join(sd, "meta.json")), dir + ": no checkpoint (neither latest nor meta.json)");
  const std::string js = read_text(join(sd, "meta.json"));
  const std::string fmt = json_value(js, "format");
  HEAT2D_REQUIRE(fmt == kFormat || fmt == kFormatV1, dir + ": not a heat2d checkpoint (" + fmt + ")");
  Meta m;
  m.dir = sd;
  m.step = std::atoll(json_value(js, "step").c_str());
  m.nranks = std::atoi(json_value(js, "nranks").c_str());
  m.dtype = json_value(js, "dtype") == "fp32" ? 0 : 1;
  m.n_owned = std::atoll(json_value(js, "n_owned").c_str());
  m.n_input = std::atoll(json_value(js, "n_input").c_str());
  m.convention = json_value(js, "convention");
  m.sigma = std::atof(json_value(js, "sigma").c_str());
  m.nu = std::atof(json_value(js, "nu").c_str());
  m.dom_len = std::atof(json_value(js, "dom_len").c_str());
  m.r = std::atof(json_value(js, "r").c_str());
  if (js.find("\"edge_shift\"") != std::string::npos) m.edge_shift = std::atoll(json_value(js, "edge_shift").c_str());
  HEAT2D_REQUIRE(m.nranks >= 1 && m.step >= 0 && m.n_owned >= 1, dir + ": inconsistent meta.json");
  return m;
}

void read_rows(const Meta& m, int64_t row0, int64_t nrows, int64_t ncols, int dtype, void* out) {
  HEAT2D_REQUIRE(dtype == m.dtype, "checkpoint dtype differs from the run's --dtype");
  const size_t es = dtype == 0 ? 4 : 8;
  int64_t start = 0;  // global row of the current writer file's first row
  for (int r = 0; r < m.nranks; ++r) {
    const std::string path = rank_file(m.dir, r);
    File file(path, "rb");
    FILE* f = file.f;
    const NpyInfo info = npy_header(f, path);
    HEAT2D_REQUIRE(info.cols == ncols && info.dtype == dtype, path + ": shape / dtype differ from the run");
    HEAT2D_REQUIRE(info.rows == decompose(m.n_owned, m.nranks, r, m.edge_shift).nrows,
                   path + ": row count differs from the writer's decomposition");
    const int64_t a = std::max(row0, start), b = std::min(row0 + nrows, start + info.rows);
    if (a < b) {
      const long off = info.data_off + (long)((a - start) * ncols * (int64_t)es);
      HEAT2D_REQUIRE(std::fseek(f, off, SEEK_SET) == 0, path + ": seek failed");
      const size_t want = (size_t)((b - a) * ncols);
      HEAT2D_REQUIRE(std::fread(static_cast<char*>(out) + (size_t)((a - row0) * ncols) * es, es, want, f) == want,
                     path + ": truncated data");
    }
    start += info.rows;
  }
  HEAT2D_REQUIRE(start == m.n_owned, m.dir + ": rank files do not cover the grid");
}

}  // namespace ckpt
}  // namespace heat2d
