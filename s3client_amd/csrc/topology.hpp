// topology.hpp -- the host's CPUs and NUMA nodes as the host path sees them: how many CPUs this
// process may use (affinity capped by the cgroup quota), how many staging threads each device
// shard gets, which node's CPUs a device's threads bind to, and the per-call thread plan
// (s3h_host_plan) that the host pipeline and the split route both follow.  HIP-free: the
// device's PCI address comes from the caller, so CPU tests drive it with a fake sysfs tree
// (S3H_SYSFS_ROOT replaces /sys) and a fake cgroup quota.
//
// MI355X nodes are dual-socket hosts with four GPUs behind each socket (the GPU box: devices
// on node 1, CPUs 64-127,192-255 local to them).  A device's DMA reads host memory through its
// socket's root complex, so the pinned staging it copies from and the threads that fill that
// staging (memcpy / pread) belong on the device's node: the sysfs numa_node and local_cpulist
// of its PCI function.  The reference's jobs run wherever the host schedules them
// (lib/src/upload.cpp:136-140 std::async, ReadFile lib/src/webclient.cpp:105-116).
#pragma once
#include <sched.h>

#include <atomic>
#include <string>
#include <vector>

namespace s3h::host {

// ------------------------------------------------------------------ CPUs
// CPU quota of this process's cgroup (v2 cpu.max, v1 cfs_quota_us / cfs_period_us), in CPUs;
// 0 when unlimited or unknown.  Read under <S3H_SYSFS_ROOT>/fs/cgroup when that is set.
double cgroup_cpu_quota();
// CPUs a process with `affinity` CPUs under a `quota` (0: none) may keep busy: the affinity
// count capped by ceil(quota), at least 1.
unsigned cpus_under(unsigned affinity, double quota);
// This process: sched_getaffinity capped by its cgroup quota (cached for the process).
unsigned host_cpus();
// Host threads (the calling thread included) each of `ndevices` concurrent device shards may
// use to stage its parts when `cpus` CPUs are available: split evenly, at least 1, at most
// kMaxStageThreads.
constexpr unsigned kMaxStageThreads = 16;
unsigned stage_threads_per_device(unsigned cpus, int ndevices);
inline unsigned host_threads_per_device(int ndevices) { return stage_threads_per_device(host_cpus(), ndevices); }
// Pageable-source staging saturates one device's H2D at >= this many threads (GPU route alone,
// profiles/r05_stage_threads_sweep.json: 2 / 4 / 6 / 8 / 16 threads 24.5 / 38.2 / 49.8 / 50.2
// / 50.5 GiB/s); fewer is reported by s3h_host_plan as below saturation.
constexpr unsigned kStageSaturation = 6;
// The split route's candidate staging threads per GPU shard for staged sources (pageable parts,
// file ranges), ascending: each device's share T / devices times 1, 4, 6, 8, 9 twelfths (at
// least 1, duplicates dropped), only those that leave the CPU side at least one thread.
std::vector<unsigned> split_stage_candidates(unsigned cpus, int ndevices);

// ------------------------------------------------------------------ NUMA (sysfs)
std::string sysfs_root();
bool read_line(const std::string& path, std::string* out);
// "0-63,128-191" -> set; false when malformed (an empty list is a valid empty set)
bool parse_cpulist(const std::string& s, cpu_set_t* set);
// sysfs NUMA record of one PCI function: node (-1 when the platform gives none) and the CPUs
// local to it.  S3H_EINVAL (last error set) when <root>/bus/pci/devices/<bdf> does not exist.
int pci_numa(const char* bdf, int* node, std::string* cpulist);
// CPUs of a NUMA node (<root>/devices/system/node/node<k>/cpulist)
bool node_cpulist(int node, std::string* cpulist);
// Node of the page holding p (get_mempolicy MPOL_F_NODE | MPOL_F_ADDR); -1 if unknown.
int mem_node(const void* p);
// Board power cap of the GPU at PCI address `bdf` in watts (<root>/bus/pci/devices/<bdf>/
// hwmon/hwmon*/power1_cap, microwatts); 0 when the platform does not say.
double pci_power_cap_w(const char* bdf);

// Placement policy: kNumaLocal (each device's node; default), kNumaOff (no binding), or a
// forced node (measurements: the remote side of an A/B).  Env S3H_HOST_NUMA = local|off|<node>.
constexpr int kNumaLocal = -1, kNumaOff = -2;
constexpr unsigned kMaxNumaNodes = 1024;
extern std::atomic<int> g_numa_mode;

// Where a device's pinned staging and threads go under the current policy: target node (-1 =
// none) and the CPUs to bind to (the node's CPUs within `affinity`; empty = unbound).
struct Place {
  int dev_node = -1;  // sysfs numa_node of the device (-1: unknown)
  int node = -1;      // staging target
  cpu_set_t cpus;
  int ncpus = 0;
  Place() { CPU_ZERO(&cpus); }
};
// Place of the device at PCI address `bdf` (null or unknown: no node) under policy `mode`,
// with `affinity` the CPUs the threads may run on (null: this thread's affinity mask).
Place place_for(const char* bdf, int mode, const cpu_set_t* affinity = nullptr);
// Binds the calling thread to P's CPUs (no-op when P has none).
void bind_self(const Place& P);

}  // namespace s3h::host
