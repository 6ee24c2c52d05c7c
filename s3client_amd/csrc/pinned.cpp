// pinned.cpp -- page-locked host memory placed on a NUMA node, device placement, and the
// pinned-ness checks the host path uses to choose between direct DMAs and staging.
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "internal.hpp"

namespace s3h::host {

namespace {

constexpr int kMpolPreferred = 1, kMpolBind = 2;

std::mutex g_reg_mu;
std::vector<std::pair<void*, size_t>>& registered_bufs() {
  static auto* v = new std::vector<std::pair<void*, size_t>>();  // never destroyed
  return *v;
}

// MemFree of a NUMA node in bytes (<root>/devices/system/node/node<k>/meminfo), -1 if unknown.
int64_t node_free_bytes(int node) {
  FILE* f = std::fopen((sysfs_root() + "/devices/system/node/node" + std::to_string(node) + "/meminfo").c_str(), "r");
  if (!f) return -1;
  char line[256];
  int64_t kb = -1;
  while (std::fgets(line, sizeof line, f))
    if (const char* p = std::strstr(line, "MemFree:")) {
      kb = std::atoll(p + 8);
      break;
    }
  std::fclose(f);
  return kb < 0 ? -1 : kb * 1024;
}

}  // namespace

// Pinned host memory whose pages live on `node`: anonymous pages placed there (mbind), touched,
// then page-locked for DMA with hipHostRegister.  node < 0: the runtime's own hipHostMalloc.
// The host path's staging PREFERS the node (MPOL_PREFERRED): when the node is short of free
// memory the kernel places the pages elsewhere instead of OOM-killing the process within the
// node, as a strict MPOL_BIND first touch would (advisor r5).  `strict` (s3h_host_alloc_ex with
// S3H_HOST_ALLOC_STRICT) binds, after checking that the node has the bytes free.
hipError_t pinned_alloc(void** out, uint64_t bytes, int node, bool strict) {
  *out = nullptr;
  if (node < 0 || node >= int(kMaxNumaNodes)) return hipHostMalloc(out, bytes, hipHostMallocDefault);
  const size_t len = std::max<size_t>(size_t(bytes), 1);
  if (strict) {  // MPOL_BIND cannot fall back: refuse what the node does not have free
    const int64_t free_b = node_free_bytes(node);
    if (free_b >= 0 && uint64_t(free_b) < len + (len >> 4) + (64ull << 20)) return hipErrorOutOfMemory;
  }
  void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return hipErrorOutOfMemory;
  unsigned long mask[kMaxNumaNodes / 64] = {};
  mask[node / 64] = 1ul << (node % 64);
  if (syscall(SYS_mbind, p, len, strict ? kMpolBind : kMpolPreferred, mask, kMaxNumaNodes + 1, 0) != 0) {
    munmap(p, len);  // node not allowed (cpuset mems) or absent: the runtime's placement
    return hipHostMalloc(out, bytes, hipHostMallocDefault);
  }
  // first touch under the policy (large buffers: 8 threads, ~0.2 s for 8 GiB instead of ~2)
  const unsigned toucher = len >= (64u << 20) ? std::min(8u, host_cpus()) : 1u;
  std::vector<std::thread> ts;
  const size_t per = (len / toucher + 4095) & ~size_t(4095);
  try {
    for (unsigned t = 1; t < toucher; ++t)
      if (t * per < len)
        ts.emplace_back([=] { std::memset(static_cast<char*>(p) + t * per, 0, std::min(per, len - t * per)); });
  } catch (const std::exception&) {  // no thread: this one touches the rest
    for (unsigned t = unsigned(ts.size()) + 1; t < toucher; ++t)
      if (t * per < len) std::memset(static_cast<char*>(p) + t * per, 0, std::min(per, len - t * per));
  }
  std::memset(p, 0, std::min(per, len));
  for (auto& th : ts) th.join();
  const hipError_t e = hipHostRegister(p, len, hipHostRegisterDefault);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    munmap(p, len);
    return e;
  }
  std::lock_guard<std::mutex> l(g_reg_mu);
  registered_bufs().push_back({p, len});
  *out = p;
  return hipSuccess;
}

void pinned_free(void* p) {
  if (!p) return;
  size_t len = 0;
  {
    std::lock_guard<std::mutex> l(g_reg_mu);
    auto& v = registered_bufs();
    for (auto it = v.begin(); it != v.end(); ++it)
      if (it->first == p) {
        len = it->second;
        v.erase(it);
        break;
      }
  }
  if (len) {
    (void)hipHostUnregister(p);
    munmap(p, len);
  } else {
    (void)hipHostFree(p);
  }
}

Place device_place(int device) {
  char bdf[32] = {0};
  if (hipDeviceGetPCIBusId(bdf, sizeof bdf, device) != hipSuccess) {
    (void)hipGetLastError();
    bdf[0] = 0;
  }
  return place_for(bdf, g_numa_mode.load());
}

bool all_pinned(const uint8_t* const* parts, const uint64_t* lengths, const uint64_t* idx, uint64_t n) {
  for (uint64_t k = 0; k < n; ++k) {
    const uint64_t i = idx ? idx[k] : k;
    if (!lengths[i]) continue;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, parts[i]) != hipSuccess || a.type != hipMemoryTypeHost) {
      (void)hipGetLastError();  // an unregistered pointer may leave a sticky error
      return false;
    }
  }
  return true;
}

// Whether [p, p + bytes) lies in ONE page-locked allocation: its first and last byte resolve to
// the same allocation range (start, size) that covers both.  A span over two separately pinned
// buffers -- with unregistered pages between them -- must not go to one DMA (advisor r5).
bool pinned_range(const void* p, uint64_t bytes) {
  if (!p || bytes == 0) return bytes == 0;
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p), hi = lo + bytes;  // [lo, hi)
  // The runtime's record of the allocation holding `a`: HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR /
  // _RANGE_SIZE answer for hipHostMalloc'd and hipHostRegister'd memory alike;
  // hipMemGetAddressRange only for the former (it returns base 0 for registered pages;
  // profiles/r06_pinned_range_probe.jsonl).
  auto range_of = [](uintptr_t a, uintptr_t* base, size_t* size) {
    void* b = nullptr;
    size_t s = 0;
    void* const p = reinterpret_cast<void*>(a);
    if (hipPointerGetAttribute(&b, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, p) == hipSuccess &&
        hipPointerGetAttribute(&s, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, p) == hipSuccess && b && s) {
      *base = reinterpret_cast<uintptr_t>(b);
      *size = s;
      return true;
    }
    (void)hipGetLastError();
    hipDeviceptr_t d = nullptr;
    if (hipMemGetAddressRange(&d, &s, reinterpret_cast<hipDeviceptr_t>(a)) == hipSuccess && d && s) {
      *base = reinterpret_cast<uintptr_t>(d);
      *size = s;
      return true;
    }
    (void)hipGetLastError();
    return false;
  };
  uintptr_t b0 = 0;
  size_t s0 = 0;
  if (range_of(lo, &b0, &s0) && lo >= b0 && hi <= b0 + s0) return true;
  // the registry of this library's own pinned buffers (pinned_alloc, s3h_host_alloc)
  std::lock_guard<std::mutex> l(g_reg_mu);
  for (const auto& r : registered_bufs()) {
    const uintptr_t rb = reinterpret_cast<uintptr_t>(r.first);
    if (lo >= rb && hi <= rb + r.second) return true;
  }
  return false;
}

}  // namespace s3h::host

using namespace s3h::host;

extern "C" {

int s3h_host_alloc_ex(int node, uint64_t bytes, int flags, void** out) {
  if (!out || bytes == 0) return fail(S3H_EINVAL, "host alloc: null out-pointer or 0 bytes");
  *out = nullptr;
  if (node < -1 || node >= int(kMaxNumaNodes)) return fail(S3H_EINVAL, "host alloc: bad node %d", node);
  if (flags & ~S3H_HOST_ALLOC_STRICT) return fail(S3H_EINVAL, "host alloc: unknown flags 0x%x", flags);
  const hipError_t e = pinned_alloc(out, bytes, node, (flags & S3H_HOST_ALLOC_STRICT) != 0);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(e == hipErrorOutOfMemory ? S3H_ENOMEM : S3H_EHIP, "host alloc (%llu B on node %d%s): %s",
                (unsigned long long)bytes, node, (flags & S3H_HOST_ALLOC_STRICT) ? ", strict" : "",
                hipGetErrorString(e));
  }
  return S3H_OK;
}

int s3h_host_alloc(int node, uint64_t bytes, void** out) { return s3h_host_alloc_ex(node, bytes, 0, out); }

int s3h_host_free(void* p) {
  pinned_free(p);
  return S3H_OK;
}

int s3h_device_numa_node(int device, int* node, char* cpulist, int len) {
  if (!node) return fail(S3H_EINVAL, "device numa: null node");
  *node = -1;
  char bdf[32];
  if (int rc = s3h_device_pci_bus_id(device, bdf, sizeof bdf)) return rc;
  return s3h_pci_numa(bdf, node, cpulist, len, nullptr);
}

}  // extern "C"
