// Persistent plan / schedule cache (plan_cache.hpp).
#include "heat2d/plan_cache.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>

#ifndef HEAT2D_BUILD_ID
#define HEAT2D_BUILD_ID "dev"
#endif

namespace heat2d {
namespace plancache {

namespace {

std::mutex g_mu;
bool g_loaded = false;
std::string g_path;
std::map<std::string, std::string> g_map;

std::string default_path() {
  if (const char* e = std::getenv("HEAT2D_PLAN_CACHE")) return e;
  std::string base;
  if (const char* x = std::getenv("XDG_CACHE_HOME"); x && *x) base = x;
  else if (const char* h = std::getenv("HOME"); h && *h) base = std::string(h) + "/.cache";
  else return "";
  return base + "/heat2d/plans-v4.txt";
}

void mkdirs(const std::string& file) {
  for (size_t p = file.find('/', 1); p != std::string::npos; p = file.find('/', p + 1))
    (void)::mkdir(file.substr(0, p).c_str(), 0755);
}

// with g_mu held
void load() {
  if (g_loaded) return;
  g_loaded = true;
  g_path = default_path();
  // a build without a source hash (HEAT2D_BUILD_ID unset: "dev") cannot tell
  // plans of older sources from its own: no cache
  if (std::string(HEAT2D_BUILD_ID) == "dev") g_path = "off";
  if (g_path.empty() || g_path == "off") return;
  std::ifstream f(g_path);
  std::string line;
  while (std::getline(f, line)) {
    const size_t t = line.find('\t');
    if (t == std::string::npos || t == 0) continue;  // torn / foreign line: ignore
    g_map[line.substr(0, t)] = line.substr(t + 1);
  }
}

bool lookup(const std::string& key, std::string* val) {
  std::lock_guard<std::mutex> g(g_mu);
  load();
  auto it = g_map.find(key);
  if (it == g_map.end()) return false;
  *val = it->second;
  return true;
}

void store(const std::string& key, const std::string& val) {
  std::lock_guard<std::mutex> g(g_mu);
  load();
  g_map[key] = val;
  if (g_path.empty() || g_path == "off") return;
  mkdirs(g_path);
  const std::string line = key + "\t" + val + "\n";
  const int fd = ::open(g_path.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
  if (fd < 0) return;  // read-only location: the cache is an optimisation only
  (void)!::write(fd, line.data(), line.size());  // one write: whole lines under O_APPEND
  ::close(fd);
}

std::string plan_key(const std::string& ctx, int k, int64_t band) {
  return "plan|" + std::string(build_id()) + "|" + ctx + "|k=" + std::to_string(k) + "|b=" + std::to_string(band);
}
std::string sched_key(const std::string& ctx, int64_t n) {
  return "sched|" + std::string(build_id()) + "|" + ctx + "|n=" + std::to_string(n);
}

}  // namespace

bool enabled() {
  std::lock_guard<std::mutex> g(g_mu);
  load();
  return !g_path.empty() && g_path != "off";
}

std::string path() {
  std::lock_guard<std::mutex> g(g_mu);
  load();
  return g_path;
}

const char* build_id() { return HEAT2D_BUILD_ID; }

void reset() {
  std::lock_guard<std::mutex> g(g_mu);
  g_loaded = false;
  g_map.clear();
  g_path.clear();
}

bool get_plan(const std::string& ctx, int k, int64_t band, kern::SplitPlan* p, float* ms) {
  std::string v;
  if (!lookup(plan_key(ctx, k, band), &v)) return false;
  std::istringstream in(v);
  kern::SplitPlan q{};
  long long r[5];
  in >> q.k >> q.ring >> q.valid >> q.nedge;
  for (auto& x : r) in >> x;
  q.main = kern::TbRect{r[0], r[1], r[2], r[3], r[4]};
  for (auto& e : q.edge) {
    for (auto& x : r) in >> x;
    e = kern::TbRect{r[0], r[1], r[2], r[3], r[4]};
  }
  long long w[4];
  for (auto& x : w) in >> x;
  q.main_waves = w[0];
  q.edge_waves = w[1];
  q.main_items = w[2];
  q.edge_items = w[3];
  float t = 0.f;
  in >> t;
  long long nr = 0;
  in >> nr;
  for (auto& e : q.rects) {
    for (auto& x : r) in >> x;
    e = kern::TbRect{r[0], r[1], r[2], r[3], r[4]};
  }
  long long pr = 0;
  in >> pr;
  q.nrects = (int32_t)nr;
  q.flags = (int32_t)pr;
  if (!in || q.k != k || q.valid < 1 || q.valid > 3 || q.nedge < 0 || q.nedge > 4 || q.nrects < 0 ||
      q.nrects > kern::kMaxPlanRects || q.flags < 0 || q.flags > (kern::kPlanDynamic | kern::kPlanLead))
    return false;
  *p = q;
  *ms = t;
  return true;
}

void put_plan(const std::string& ctx, int k, int64_t band, const kern::SplitPlan& p, float ms) {
  std::ostringstream o;
  o << p.k << ' ' << p.ring << ' ' << p.valid << ' ' << p.nedge;
  auto rect = [&](const kern::TbRect& R) { o << ' ' << R.r0 << ' ' << R.r1 << ' ' << R.s0 << ' ' << R.s1 << ' ' << R.nb; };
  rect(p.main);
  for (const auto& e : p.edge) rect(e);
  o << ' ' << p.main_waves << ' ' << p.edge_waves << ' ' << p.main_items << ' ' << p.edge_items << ' ' << ms;
  o << ' ' << p.nrects;
  for (const auto& e : p.rects) rect(e);
  o << ' ' << p.flags;
  store(plan_key(ctx, k, band), o.str());
}

bool get_schedule(const std::string& ctx, int64_t n, std::vector<int>* sched) {
  std::string v;
  if (!lookup(sched_key(ctx, n), &v)) return false;
  std::istringstream in(v);
  std::vector<int> s;
  int d;
  int64_t sum = 0;
  while (in >> d) {
    if (d < 1) return false;
    s.push_back(d);
    sum += d;
  }
  if (s.empty() || sum != n) return false;
  *sched = std::move(s);
  return true;
}

void put_schedule(const std::string& ctx, int64_t n, const std::vector<int>& sched) {
  std::ostringstream o;
  for (size_t i = 0; i < sched.size(); ++i) o << (i ? " " : "") << sched[i];
  store(sched_key(ctx, n), o.str());
}

}  // namespace plancache
}  // namespace heat2d
