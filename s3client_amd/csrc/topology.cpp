// topology.cpp -- CPUs, NUMA nodes and the host thread plan (topology.hpp), and the C-ABI
// entry points that need no GPU: s3h_host_threads, s3h_host_plan, s3h_pci_numa, s3h_mem_node.
#include "topology.hpp"

#include <dirent.h>
#include <pthread.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "../../include/s3hash.h"
#include "status.hpp"

namespace s3h::host {

// ------------------------------------------------------------------ CPUs
// The reference's jobs run as std::async threads on whatever the host grants
// (lib/src/upload.cpp:136-140); hardware_concurrency() counts the machine's CPUs instead --
// 256 on the GPU box, whose container quota is 16, where over-subscribed copy threads halved
// the staging rate (BENCH_r02 cpu_baseline.GiBps_by_threads).
double cgroup_cpu_quota() {
  const std::string cg = sysfs_root() + "/fs/cgroup";
  double q = 0, per = 0;
  if (FILE* f = std::fopen((cg + "/cpu.max").c_str(), "r")) {
    char a[32] = {0};
    const int got = std::fscanf(f, "%31s %lf", a, &per);
    std::fclose(f);
    if (got == 2 && std::strcmp(a, "max") != 0 && per > 0) return std::atof(a) / per;
    if (got >= 1) return 0;  // "max": unlimited
  }
  FILE* fq = std::fopen((cg + "/cpu/cpu.cfs_quota_us").c_str(), "r");
  FILE* fp = std::fopen((cg + "/cpu/cpu.cfs_period_us").c_str(), "r");
  const bool ok = fq && fp && std::fscanf(fq, "%lf", &q) == 1 && std::fscanf(fp, "%lf", &per) == 1 &&
                  q > 0 && per > 0;
  if (fq) std::fclose(fq);
  if (fp) std::fclose(fp);
  return ok ? q / per : 0;
}

unsigned cpus_under(unsigned affinity, double quota) {
  unsigned n = std::max(1u, affinity);
  if (quota > 0) n = std::min(n, std::max(1u, unsigned(std::ceil(quota))));
  return n;
}

unsigned host_cpus() {
  static const unsigned cpus = [] {
    unsigned n = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0 && CPU_COUNT(&set) > 0) n = unsigned(CPU_COUNT(&set));
    return cpus_under(n, cgroup_cpu_quota());
  }();
  return cpus;
}

unsigned stage_threads_per_device(unsigned cpus, int ndevices) {
  return std::min(kMaxStageThreads, std::max(1u, cpus / unsigned(std::max(1, ndevices))));
}

std::vector<unsigned> split_stage_candidates(unsigned cpus, int ndevices) {
  const unsigned devs = unsigned(std::max(1, ndevices));
  const unsigned share = std::max(1u, cpus / devs);
  std::vector<unsigned> cand;
  for (unsigned num : {1u, 4u, 6u, 8u, 9u}) {  // x share / 12: share/12 ... 3 share/4
    const unsigned t = std::max(1u, share * num / 12);
    if (uint64_t(t) * devs < cpus && std::find(cand.begin(), cand.end(), t) == cand.end()) cand.push_back(t);
  }
  return cand;
}

// ------------------------------------------------------------------ NUMA (sysfs)
constexpr int kMpolFNode = 1, kMpolFAddr = 2;

std::string sysfs_root() {
  const char* e = std::getenv("S3H_SYSFS_ROOT");
  return e && *e ? std::string(e) : std::string("/sys");
}

bool read_line(const std::string& path, std::string* out) {
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) return false;
  char buf[4096];
  const bool ok = std::fgets(buf, sizeof buf, f) != nullptr;
  std::fclose(f);
  if (!ok) return false;
  *out = buf;
  while (!out->empty() && std::isspace(static_cast<unsigned char>(out->back()))) out->pop_back();
  return true;
}

bool parse_cpulist(const std::string& s, cpu_set_t* set) {
  CPU_ZERO(set);
  const char* p = s.c_str();
  while (*p) {
    char* end = nullptr;
    const long a = std::strtol(p, &end, 10);
    if (end == p || a < 0) return false;
    long b = a;
    p = end;
    if (*p == '-') {
      b = std::strtol(p + 1, &end, 10);
      if (end == p + 1 || b < a) return false;
      p = end;
    }
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET(int(c), set);
    if (*p == ',') ++p;
    else if (*p) return false;
  }
  return true;
}

int pci_numa(const char* bdf, int* node, std::string* cpulist) {
  if (!bdf || !*bdf) return fail(S3H_EINVAL, "pci numa: empty PCI address");
  std::string b(bdf);
  for (char& c : b) c = char(std::tolower(static_cast<unsigned char>(c)));
  const std::string dir = sysfs_root() + "/bus/pci/devices/" + b;
  std::string v;
  if (!read_line(dir + "/numa_node", &v))
    return fail(S3H_EINVAL, "pci numa: cannot read %s/numa_node", dir.c_str());
  *node = std::atoi(v.c_str());
  if (*node < 0) *node = -1;
  if (!read_line(dir + "/local_cpulist", cpulist)) cpulist->clear();
  return S3H_OK;
}

bool node_cpulist(int node, std::string* cpulist) {
  return node >= 0 && read_line(sysfs_root() + "/devices/system/node/node" + std::to_string(node) + "/cpulist", cpulist);
}

int mem_node(const void* p) {
  int node = -1;
  if (!p || syscall(SYS_get_mempolicy, &node, nullptr, 0, p, kMpolFNode | kMpolFAddr) != 0) return -1;
  return node;
}

double pci_power_cap_w(const char* bdf) {
  if (!bdf || !*bdf) return 0;
  std::string b(bdf);
  for (char& c : b) c = char(std::tolower(static_cast<unsigned char>(c)));
  const std::string dir = sysfs_root() + "/bus/pci/devices/" + b + "/hwmon";
  DIR* d = opendir(dir.c_str());
  if (!d) return 0;
  double w = 0;
  while (dirent* e = readdir(d)) {
    if (std::strncmp(e->d_name, "hwmon", 5) != 0) continue;
    std::string v;
    if (read_line(dir + "/" + e->d_name + "/power1_cap", &v) && std::atof(v.c_str()) > 0) {
      w = std::atof(v.c_str()) * 1e-6;
      break;
    }
  }
  closedir(d);
  return w;
}

std::atomic<int> g_numa_mode{[] {
  const char* e = std::getenv("S3H_HOST_NUMA");
  if (!e || !*e || std::strcmp(e, "local") == 0) return kNumaLocal;
  if (std::strcmp(e, "off") == 0) return kNumaOff;
  return std::isdigit(static_cast<unsigned char>(e[0])) ? std::atoi(e) : kNumaLocal;
}()};

Place place_for(const char* bdf, int mode, const cpu_set_t* affinity) {
  Place P;
  std::string local;
  if (bdf && *bdf) {
    const std::string saved = g_err;  // a device without a sysfs record is not an error here
    if (pci_numa(bdf, &P.dev_node, &local) != S3H_OK) {
      P.dev_node = -1;
      local.clear();
    }
    g_err = saved;
  }
  if (mode == kNumaOff) return P;
  P.node = mode == kNumaLocal ? P.dev_node : mode;
  if (P.node < 0) return P;
  std::string list = mode == kNumaLocal ? local : std::string();
  if (list.empty()) node_cpulist(P.node, &list);
  cpu_set_t want, mine;
  if (!parse_cpulist(list, &want)) return P;
  if (affinity) mine = *affinity;
  else if (sched_getaffinity(0, sizeof mine, &mine) != 0) return P;
  (void)CPU_AND(&P.cpus, &want, &mine);
  P.ncpus = CPU_COUNT(&P.cpus);
  return P;
}

void bind_self(const Place& P) {
  if (P.ncpus > 0) (void)pthread_setaffinity_np(pthread_self(), sizeof P.cpus, &P.cpus);
}

}  // namespace s3h::host

using namespace s3h::host;

extern "C" {

int s3h_host_threads(int ndevices, int* cpus) {
  if (cpus) *cpus = int(host_cpus());
  return int(host_threads_per_device(ndevices));
}

int s3h_host_plan(const char* const* pci_bus_ids, int ndevices, const char* affinity_cpulist,
                  double cpu_quota, s3h_host_plan_t* plan, s3h_host_plan_device_t* devices) {
  if (!plan || ndevices <= 0 || ndevices > 4096)
    return fail(S3H_EINVAL, "host plan: need a plan and 1 <= ndevices <= 4096");
  *plan = s3h_host_plan_t{};
  cpu_set_t aff;
  if (affinity_cpulist) {
    if (!parse_cpulist(affinity_cpulist, &aff) || CPU_COUNT(&aff) == 0)
      return fail(S3H_EINVAL, "host plan: bad affinity list \"%s\"", affinity_cpulist);
  } else if (sched_getaffinity(0, sizeof aff, &aff) != 0) {
    return fail(S3H_EINVAL, "host plan: sched_getaffinity failed");
  }
  const double quota = cpu_quota < 0 ? cgroup_cpu_quota() : cpu_quota;
  const unsigned cpus = cpus_under(unsigned(CPU_COUNT(&aff)), quota);
  const unsigned per = stage_threads_per_device(cpus, ndevices);
  plan->cpus = int(cpus);
  plan->affinity_cpus = CPU_COUNT(&aff);
  plan->cpu_quota = quota;
  plan->devices = ndevices;
  plan->staging_threads_per_device = int(per);
  plan->threads = int(per) * ndevices;
  plan->oversubscribed = plan->threads > int(cpus);
  plan->below_saturation = per < kStageSaturation;
  plan->split_cpu_threads_pinned = int(cpus);  // pinned parts: DMAs, every thread to the CPU side
  const std::vector<unsigned> cand = split_stage_candidates(cpus, ndevices);
  plan->split_candidates = int(cand.size());
  if (!cand.empty()) {
    plan->split_stage_min = int(cand.front());
    plan->split_stage_max = int(cand.back());
    plan->split_cpu_threads_max = int(cpus - cand.front() * unsigned(ndevices));
    plan->split_cpu_threads_min = int(cpus - cand.back() * unsigned(ndevices));
  }
  // threads bound to each node vs the CPUs they may bind to there
  std::vector<std::pair<int, int>> node_load;  // (node, threads)
  std::vector<int> node_cpus;
  for (int d = 0; d < ndevices; ++d) {
    const char* bdf = pci_bus_ids ? pci_bus_ids[d] : nullptr;
    const Place P = place_for(bdf, g_numa_mode.load(), &aff);
    if (devices) {
      s3h_host_plan_device_t& D = devices[d];
      D = s3h_host_plan_device_t{};
      D.node = P.dev_node;
      D.bind_node = P.ncpus > 0 ? P.node : -1;
      D.bind_cpus = P.ncpus;
      D.staging_threads = int(per);
      int first = -1, last = -1;
      for (int c = 0; c < CPU_SETSIZE; ++c)
        if (CPU_ISSET(c, &P.cpus)) {
          if (first < 0) first = c;
          last = c;
        }
      D.bind_first_cpu = first;
      D.bind_last_cpu = last;
    }
    if (P.ncpus <= 0) continue;
    size_t k = 0;
    while (k < node_load.size() && node_load[k].first != P.node) ++k;
    if (k == node_load.size()) {
      node_load.push_back({P.node, 0});
      node_cpus.push_back(P.ncpus);
    }
    node_load[k].second += int(per);
    node_cpus[k] = std::min(node_cpus[k], P.ncpus);
  }
  for (size_t k = 0; k < node_load.size(); ++k)
    if (node_load[k].second > node_cpus[k]) plan->node_oversubscribed = 1;
  return S3H_OK;
}

int s3h_pci_power_cap(const char* pci_bus_id, double* watts) {
  if (!pci_bus_id || !watts) return fail(S3H_EINVAL, "pci power cap: null argument");
  *watts = pci_power_cap_w(pci_bus_id);
  return S3H_OK;
}

int s3h_pci_numa(const char* pci_bus_id, int* node, char* cpulist, int len, int* usable_cpus) {
  if (!node) return fail(S3H_EINVAL, "pci numa: null node");
  *node = -1;
  if (cpulist && len > 0) cpulist[0] = 0;
  if (usable_cpus) *usable_cpus = 0;
  std::string local;
  if (int rc = pci_numa(pci_bus_id, node, &local)) return rc;
  if (cpulist && len > 0) std::snprintf(cpulist, size_t(len), "%s", local.c_str());
  cpu_set_t want, mine, both;
  if (usable_cpus && parse_cpulist(local, &want) && sched_getaffinity(0, sizeof mine, &mine) == 0) {
    (void)CPU_AND(&both, &want, &mine);
    *usable_cpus = CPU_COUNT(&both);
  }
  return S3H_OK;
}

int s3h_mem_node(const void* p, int* node) {
  if (!p || !node) return fail(S3H_EINVAL, "mem node: null argument");
  *node = mem_node(p);
  return *node >= 0 ? S3H_OK : fail(S3H_EINVAL, "mem node: get_mempolicy failed (%s)", std::strerror(errno));
}

}  // extern "C"
