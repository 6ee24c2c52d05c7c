/* include/s3hash.h -- C-ABI of the MI355X batched SHA-256 path (libs3hash.so).
 *
 * This is the boundary the S3 client links against for PAYLOAD hashing: plain pointers and
 * sizes, int status codes, no C++ or HIP types, no exceptions.  It sits beside the C++
 * drop-in of lib/hash (include/sha256.h, include/utility.h), whose single-message calls stay
 * on the CPU exactly as in the reference.
 *
 * Reference interfaces each entry point serves (paths under /root/reference):
 *   s3h_sha256_batch_device / s3h_plan_*  -- batched form of sha256::sha256
 *       (lib/hash/sha256.h:70, lib/hash/sha256.cpp:147-160), applied to the parts that
 *       lib/src/upload.cpp:89-110 (UploadParts) slices, before each part's digest is passed
 *       as `payloadHash` to S3Api::UploadFilePart (lib/include/s3-api.h:447-452).
 *   s3h_sha256_batch_host  -- the same starting and ending in host memory (file chunks
 *       staged for upload -> 32-byte digests handed back to the SigV4 signer,
 *       lib/src/aws_sign.cpp:236-237 x-amz-content-sha256).
 *   s3h_plan_launch_range  -- resumable chaining state: sha256::sha256_stream semantics
 *       (lib/hash/sha256.h:97, sha256.cpp:84-144) for many parts at once.
 *
 * Digest layout (every entry point): 8 uint32 words per part with word i = bswap32(H_i),
 * exactly lib/hash's `to_little` output (sha256.h:103-106); on little-endian hosts the 32
 * bytes in memory are the canonical SHA-256 digest, and sha256::hash_to_text prints them.
 */
#ifndef S3HASH_H
#define S3HASH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: s3h_route_rates_t / s3h_route_choose (size-carrying, digest sets), s3h_host_plan,
 * s3h_host_alloc_ex, MD5 and dual routed entry points.  s3h_route_model_t keeps its round-5
 * layout (8 fields) for good: new rates go to s3h_route_rates_t, which carries its size. */
#define S3H_API_VERSION 2

enum s3h_status {
  S3H_OK = 0,
  S3H_EINVAL = -1,   /* bad argument (null pointer, bad device, n too large, ...) */
  S3H_ENODEV = -2,   /* no HIP device visible: the GPU path never falls back to the CPU */
  S3H_EHIP = -3,     /* HIP runtime error (message in s3h_last_error) */
  S3H_ENOMEM = -4    /* device or pinned host allocation failed */
};

enum s3h_kernel {
  S3H_KERNEL_AUTO = 0, /* choose by part count */
  S3H_KERNEL_LANE = 1, /* fused: one lane = schedule + rounds of one part */
  S3H_KERNEL_PC = 2,   /* producer/consumer: producer wave stages W+K through LDS */
  S3H_KERNEL_PAIR = 3, /* producer/consumer with each chain split over a lane pair (DPP) */
  S3H_KERNEL_QUAD = 4, /* as PAIR, each half-state on a lane quad: 9 instead of 10 VALU/round */
  S3H_KERNEL_SKEW = 5, /* lane quads with the a-quad two rounds behind: 8 VALU/round */
  S3H_KERNEL_SKEWP = 6, /* the same skewed schedule on lane pairs: 9 VALU/round, 32 chains/wave */
  S3H_KERNEL_SKEWS = 7  /* SKEW with each producer on its consumer's SIMD: 32 chains per CU */
};

enum s3h_algo {
  S3H_ALGO_SHA256 = 0, /* payload SHA-256 (x-amz-content-sha256), digests n x 8 words */
  S3H_ALGO_MD5 = 1     /* MD5 (Content-MD5, multipart ETags), digests n x 4 words */
};

/* What AUTO optimises when several kernels fit a batch (s3h_kernel_policy).  They differ only
 * for 4,097 - 32 x CUs parts (8,192 on MI355X: the C4 shard), where the shared-SIMD SKEWS
 * kernel is ~5 % faster than SKEWP but draws 1.26-1.34 kW against 0.77 kW (2.57 vs 1.65 J/GiB):
 * S3H_POLICY_THROUGHPUT -- SKEWS; S3H_POLICY_EFFICIENCY -- SKEWP (the lower energy-delay
 * product); S3H_POLICY_POWER (default since API 2) -- SKEWS only when the device's board power
 * cap (sysfs hwmon power1_cap, s3h_device_power_cap) lets it hold its full clock (>= 1,500 W:
 * consumers and producers together need ~1.52 kW, more than MI355X's 1,400 W cap), SKEWP
 * otherwise.  Initial value from the environment: S3H_KERNEL_POLICY=throughput|efficiency|power
 * (S3H_PREFER_EFFICIENCY=1 = efficiency). */
enum s3h_policy { S3H_POLICY_THROUGHPUT = 0, S3H_POLICY_EFFICIENCY = 1, S3H_POLICY_POWER = 2 };

/* Last error message of the calling thread ("" if none). */
const char *s3h_last_error(void);
int s3h_api_version(void);
/* Free the host path's cached per-device contexts.  Between s3h_*_batch_host /
 * s3h_sha256_file_parts / s3h_verify_batch_host calls each device keeps one context:
 * streams, plans, digest buffers, copy threads, at most 1 GiB of HBM ring (larger rings are
 * freed when the call returns) and its pinned staging (96 MiB, up to 384 MiB after a
 * file-range call with thousands of parts).  Concurrent host calls on one device are merged
 * into one batch (their digests are the same as from separate calls).  s3h_trim releases the
 * contexts of idle devices. */
int s3h_trim(void);
/* Set AUTO's kernel policy for plans created afterwards (initially S3H_POLICY_POWER, see
 * above); *previous receives the old one.  No GPU. */
int s3h_kernel_policy(int policy, int *previous);
/* Board power cap of HIP device `device` in watts as the POWER policy reads it (0: unknown). */
int s3h_device_power_cap(int device, double *watts);
/* Host threads (the calling thread included) the host path uses per device to stage
 * pageable parts and file ranges when `ndevices` device shards run at once: the CPUs this
 * process may use -- its sched_getaffinity mask, capped by the cgroup CPU quota (cpu.max, or
 * cfs_quota_us / cfs_period_us) -- split evenly over the devices, at least 1 and at most 16.
 * *cpus (if non-null) receives that CPU count.  Needs no GPU.  The reference's jobs run on
 * the cores the host grants (lib/src/upload.cpp:136-140, std::async). */
int s3h_host_threads(int ndevices, int *cpus);
/* The host path's thread plan for a call over `ndevices` devices at PCI addresses
 * pci_bus_ids[k] (null entries or a null array: no NUMA record), with the CPUs of
 * `affinity_cpulist` ("0-63,128-191"; null: this process's affinity) under a cgroup quota of
 * `cpu_quota` CPUs (0: none; < 0: this process's quota) -- pure host arithmetic over sysfs
 * (S3H_SYSFS_ROOT replaces /sys), the rules the host pipeline and the split route apply, so an
 * N-GPU host can be checked before it runs:
 *   staging threads per device = min(16, max(1, cpus / ndevices)), each device's threads bound
 *   to its node's CPUs within the affinity; the split route from pinned parts gives the CPU side
 *   every thread, from staged sources each device tg of its share (1, 4, 6, 8, 9 twelfths) and
 *   the CPU side the rest.  devices (if non-null) receives ndevices records. */
typedef struct {
  int cpus;                       /* affinity capped by ceil(quota) */
  int affinity_cpus;
  double cpu_quota;               /* the quota applied (0: none) */
  int devices;
  int staging_threads_per_device; /* host threads staging one device's pageable parts / files */
  int threads;                    /* staging threads of the whole call */
  int oversubscribed;             /* threads > cpus (ndevices > cpus: one thread each anyway) */
  int below_saturation;           /* per-device staging < 6 threads: pageable sources below the
                                     H2D rate of one device (profiles/r05_stage_threads_sweep.json) */
  int node_oversubscribed;        /* some node's bound threads exceed its bindable CPUs */
  int split_cpu_threads_pinned;   /* split route, pinned parts: the CPU side's threads */
  int split_candidates;           /* split route, staged sources: staging-thread choices (0: none fits) */
  int split_stage_min, split_stage_max;            /* per device */
  int split_cpu_threads_min, split_cpu_threads_max; /* the CPU side's threads at those choices */
} s3h_host_plan_t;
typedef struct {
  int node;            /* sysfs numa_node (-1: unknown) */
  int bind_node;       /* node its threads and staging go to (-1: unbound) */
  int bind_cpus;       /* CPUs its shard / copy threads bind to (0: unbound) */
  int bind_first_cpu;  /* lowest and highest of them (-1: none) */
  int bind_last_cpu;
  int staging_threads;
} s3h_host_plan_device_t;
int s3h_host_plan(const char *const *pci_bus_ids, int ndevices, const char *affinity_cpulist,
                  double cpu_quota, s3h_host_plan_t *plan, s3h_host_plan_device_t *devices);
/* Number of visible HIP devices; S3H_ENODEV (and *count = 0) when there is none. */
int s3h_device_count(int *count);
/* PCI address of HIP device `device` as "dddd:bb:dd.f" (lowercase, NUL-terminated; len >= 13):
 * which physical GPU a device index names, so a multi-GPU run can show that its N ranks
 * hashed on N distinct devices.  S3H_ENODEV / S3H_EINVAL as s3h_plan_create. */
int s3h_device_pci_bus_id(int device, char *out, int len);

/* ---------------------------------------------------------------- NUMA placement
 * MI355X hosts are dual-socket with four GPUs behind each socket.  The host path puts each
 * device's pinned staging (pageable parts, file ranges, stream bookkeeping) on the device's
 * NUMA node and binds its copy threads -- and, for multi-device calls, each device's shard
 * thread -- to that node's CPUs within the process's affinity mask.  The reference's upload
 * jobs run wherever the host schedules them (lib/src/upload.cpp:136-140, std::async; bytes
 * read by ReadFile, lib/src/webclient.cpp:105-116).  None of these needs a GPU except where
 * stated; S3H_SYSFS_ROOT (tests) replaces /sys.
 *
 * NUMA record of a PCI function "dddd:bb:dd.f": sysfs numa_node (-1 when the platform gives
 * none), local_cpulist (into cpulist, NUL-terminated, truncated to len) and how many of those
 * CPUs this thread's affinity mask allows.  S3H_EINVAL when the function has no sysfs entry. */
int s3h_pci_numa(const char *pci_bus_id, int *node, char *cpulist, int len, int *usable_cpus);
/* The same for HIP device `device` (needs the device: its PCI address). */
int s3h_device_numa_node(int device, int *node, char *cpulist, int len);
/* Board power cap of the PCI function in watts (sysfs hwmon<k>/power1_cap; 0 when the platform
 * does not report one): what S3H_POLICY_POWER reads for a device.  No GPU needed. */
int s3h_pci_power_cap(const char *pci_bus_id, double *watts);
/* Placement policy of the host path: S3H_NUMA_LOCAL (default: each device's own node),
 * S3H_NUMA_OFF (no binding: the runtime's placement, unbound threads) or a node >= 0 (every
 * device's staging and threads on that node -- for local/remote measurements).  Initial value
 * from the environment: S3H_HOST_NUMA=local|off|<node>.  Idle cached contexts are released
 * so the next call re-places them.  *previous (if non-null) receives the old mode. */
#define S3H_NUMA_LOCAL (-1)
#define S3H_NUMA_OFF (-2)
int s3h_host_numa(int mode, int *previous);
typedef struct {
  int device_node;  /* sysfs numa_node of the device (-1: unknown) */
  int target_node;  /* node the policy places its staging on (-1: none) */
  int bound_cpus;   /* CPUs its copy / shard threads bind to (0: unbound) */
  int staging_node; /* measured node of the cached context's staging ring (-1: none yet) */
  int threads_node; /* node the cached context's copy threads are bound to (-1: unbound/none) */
  int copy_threads; /* copy threads of the cached context (0: none yet) */
} s3h_host_numa_t;
/* Placement of device `device` under the current policy, plus what its cached host context
 * actually holds (needs the device). */
int s3h_host_numa_info(int device, s3h_host_numa_t *info);
/* Pinned (page-locked, DMA-able) host memory whose pages are bound to NUMA node `node`
 * (-1: the runtime's placement): an uploader's read buffers on its device's node.  Needs a
 * HIP device.  Free with s3h_host_free. */
int s3h_host_alloc(int node, uint64_t bytes, void **out);
/* The same with flags.  Default (and s3h_host_alloc): the node is PREFERRED -- when it is short
 * of free memory the pages go to another node instead of the process being OOM-killed within
 * the node.  S3H_HOST_ALLOC_STRICT binds the pages to the node (MPOL_BIND) after checking that
 * the node has the bytes free (S3H_ENOMEM otherwise). */
#define S3H_HOST_ALLOC_STRICT 1
int s3h_host_alloc_ex(int node, uint64_t bytes, int flags, void **out);
int s3h_host_free(void *p);
/* NUMA node of the page holding host address p (get_mempolicy). */
int s3h_mem_node(const void *p, int *node);

/* ---------------------------------------------------------------- device-resident path
 * A plan captures the part geometry (byte offsets relative to a base pointer, lengths) of
 * one batch, sorted on the host by block count and uploaded once to `device`.  Launching it
 * hashes every part of a device buffer laid out that way; the same plan can be launched on
 * many buffers with that layout.  `stream` is a hipStream_t (NULL = the null stream). */
typedef struct s3h_plan_s *s3h_plan_t;

int s3h_plan_create(int device, const uint64_t *offsets, const uint64_t *lengths, uint64_t n,
                    int kernel, s3h_plan_t *plan);
/* Same for any algorithm (s3h_algo); digests are 8 (SHA-256) or 4 (MD5) words per part. */
int s3h_plan_create_ex(int device, int algo, const uint64_t *offsets, const uint64_t *lengths,
                       uint64_t n, int kernel, s3h_plan_t *plan);
int s3h_plan_algo(s3h_plan_t plan);
int s3h_plan_destroy(s3h_plan_t plan);
/* Asynchronous on `stream`: d_base and d_digests (n*8 uint32) are device pointers.  The
 * launch's success is known only after it has run: call s3h_plan_status before using the
 * digests. */
int s3h_plan_launch(s3h_plan_t plan, const void *d_base, uint32_t *d_digests, void *stream);
/* Waits for `stream`, then reads and clears the plan's device error word, which every launch
 * of the plan (s3h_plan_launch / _range) ORs its faults into.  S3H_OK: the digests of every
 * launch since the last status call are valid.  S3H_EHIP ("synchronisation timeout"): a
 * flag-synchronised kernel (the two-group skew, shared-SIMD skew and dual-digest group
 * kernels pair a producer and a consumer wave through LDS step counters) gave up a bounded
 * wait, so the grid drained instead of hanging and those digests are NOT the parts' digests.
 * The one-shot, host, dual, verification and stream entry points check this word themselves
 * and fail the call; lib/hash's sha256() (sha256.cpp:147-160) never returns a wrong digest. */
int s3h_plan_status(s3h_plan_t plan, void *stream);
/* Resumable form: process blocks [blk_begin, blk_end) of every part, where part p's block b
 * lives at d_base + offsets[p] + 64*(b - blk_origin).  Chaining state is kept in the plan
 * between launches (same stream order required); a part's digest is written by the launch
 * that processes its final (padding) block. */
int s3h_plan_launch_range(s3h_plan_t plan, const void *d_base, uint32_t *d_digests,
                          uint64_t blk_begin, uint64_t blk_end, uint64_t blk_origin,
                          void *stream);
/* Introspection: total 64-B compressions, max blocks of any part, chosen kernel, grid size. */
int s3h_plan_info(s3h_plan_t plan, uint64_t *n, uint64_t *total_blocks, uint64_t *max_blocks,
                  int *kernel, uint32_t *grid);
/* Workgroup layout: consumer groups of the grid (skew/skewp kernels; 0 for the others) and how
 * many leading workgroups of the two-group skew kernel run one group on a CU of their own
 * (the groups of the longest parts of a ragged batch). */
int s3h_plan_groups(s3h_plan_t plan, uint32_t *groups, uint32_t *solo);
/* SHA-256 + MD5 of a SHA-256 plan's parts (s3h_sha256_md5_batch_*): how many leading
 * workgroups of the one-grid dual kernel run the longest parts as 8-part skew groups (a
 * ragged batch of 2,049 - 32 x CUs parts); 0 when the dual pass uses another form. */
int s3h_plan_dual_solo(s3h_plan_t plan, uint32_t *solo);
/* The same plus which form of that mixed grid runs: *apart = 1 when the skew groups' MD5
 * chains run on workgroups of their own (round 4, each skew group at the SHA-256-alone rate),
 * 0 when each skew group carries its MD5 wave (round 3; used when the apart grid would exceed
 * one workgroup per CU). */
int s3h_plan_dual_layout(s3h_plan_t plan, uint32_t *solo, int *apart);
/* That choice for a batch of `lengths` on a device of `cus` CUs, without a device (pure host
 * arithmetic, the rule the plan applies). */
int s3h_dual_layout(const uint64_t *lengths, uint64_t n, int cus, uint32_t *solo, int *apart);

/* Measurement hook (not part of the lib/hash surface): while d_clocks (device memory,
 * 4 x *waves uint64) is set, every launch of a plan on the skew kernel records, per consumer
 * wave, the shader-clock counter (s_memtime) and the 100 MHz real-time counter
 * (s_memrealtime) at the start and end of its chain loop: {clk0, clk1, rt0, rt1}.  *waves
 * receives the number of consumer waves (0: the plan's kernel does not record).  NULL turns
 * the probe off.  bench.py uses it to report cycles per block and the live shader clock. */
int s3h_plan_set_clock_probe(s3h_plan_t plan, uint64_t *d_clocks, uint32_t *waves);

/* One-shot convenience: plan + launch + wait.  Returns when d_digests is complete. */
int s3h_sha256_batch_device(int device, const void *d_base, const uint64_t *offsets,
                            const uint64_t *lengths, uint64_t n, uint32_t *d_digests,
                            void *stream);

/* Batched MD5 (lib/hash/md5.cpp semantics with md5_file's padding): n x 4 words, the
 * digest bytes in memory order (md5::hash_to_text prints them). */
int s3h_md5_batch_device(int device, const void *d_base, const uint64_t *offsets,
                         const uint64_t *lengths, uint64_t n, uint32_t *d_digests, void *stream);

/* ---------------------------------------------------------------- host-resident path
 * parts[i] (host memory, pinned or pageable) of lengths[i] bytes -> digests (host, n*8).
 * Parts are sharded round-robin over `ndevices` GPUs (0 = all visible), part i on device
 * i % ndevices; each device streams its parts through HBM in slices of `slice_bytes` per
 * part with copies overlapped with hashing.  slice_bytes 0 = auto: pinned parts are DMA'd
 * directly (256 KiB slices and one 2-D copy per slice when they are equal-length chunks at a
 * constant host stride, 2 MiB per-part copies otherwise); pageable parts (e.g. an mmap'd
 * file) are first copied by host threads into a pinned staging ring (at most 32 MiB per
 * slot: slices of 32 MiB / n bytes, down to 64 B) and DMA'd from there; beyond 524,288
 * pageable parts, or when pinned memory is unavailable, each part is DMA'd from pageable memory.
 * Everything is cached per device between calls (s3h_trim).  Safe to call from concurrent
 * threads (concurrent calls on a device are merged into one batch, see
 * s3h_sha256_batch_host_on).  Blocking. */
int s3h_sha256_batch_host(const uint8_t *const *parts, const uint64_t *lengths, uint64_t n,
                          uint32_t *digests, int ndevices, uint64_t slice_bytes);

int s3h_md5_batch_host(const uint8_t *const *parts, const uint64_t *lengths, uint64_t n,
                       uint32_t *digests, int ndevices, uint64_t slice_bytes);

/* The same over an explicit device list: shard k = parts i with i % ndevices == k, hashed on
 * devices[k].  A device may be listed more than once: its shards then meet in that device's
 * queue like concurrent callers (below) and run merged into one batch, or one after another
 * when they arrive apart -- the digests are the same either way (this is how the sharding is
 * exercised on a one-GPU host).  Concurrent host calls on one device are merged in its queue:
 * the first caller runs every pending request with the same algorithms and slice size as one
 * batch; if that batch fails, each request is re-run on its own, so each caller gets its own
 * status.  Staging threads per device: s3h_host_threads(number of shards). */
int s3h_sha256_batch_host_on(const uint8_t *const *parts, const uint64_t *lengths, uint64_t n,
                             uint32_t *digests, const int *devices, int ndevices,
                             uint64_t slice_bytes);

/* Parts given as byte ranges of a file: part i = [offsets[i], offsets[i] + lengths[i]) of
 * `path` -- the (file, offset, size) parts that S3Api::UploadFilePart sends
 * (lib/src/api/multipart_upload.cpp:216-223 -> WebClient::UploadFile, webclient.cpp:331-355),
 * i.e. a batched sha256::sha256_file (lib/hash/sha256.cpp:183-233) over ranges.  Host threads
 * pread each slice straight into the pinned staging ring (no intermediate copy); its slots
 * are 128 MiB (32 KiB slices up to 4,096 parts per device), so the per-slice syscall does not
 * dominate.
 * S3H_EINVAL when the file cannot be opened or is shorter than a part.  Blocking. */
int s3h_sha256_file_parts(const char *path, const uint64_t *offsets, const uint64_t *lengths,
                          uint64_t n, uint32_t *digests, int ndevices, uint64_t slice_bytes);

/* ---------------------------------------------------------------- dual digest
 * x-amz-content-sha256 AND Content-MD5 of every part in one call (an upload that sends both
 * headers; the MD5s also give the multipart ETag).  Replaces a sha256::sha256 plus an
 * md5::md5 call per part (lib/hash/sha256.cpp:147-160, lib/hash/md5.cpp:71-180).
 * Both forms launch ONE grid whose workgroups run either the SHA-256 or the MD5 chain
 * (sha256_md5_dual_kernel) while it fits one workgroup per CU, so both digests take the
 * SHA-256 time; larger batches (> 32 x CUs parts, where each kernel fills the chip) run the
 * two kernels one after the other.  Host form: each slice
 * crosses PCIe ONCE for both digests (the host path is PCIe-bound).  Blocking.
 * sha256_digests: n x 8 words (lib/hash layout); md5_digests: n x 4 words (memory order). */
int s3h_sha256_md5_batch_host(const uint8_t *const *parts, const uint64_t *lengths, uint64_t n,
                              uint32_t *sha256_digests, uint32_t *md5_digests, int ndevices,
                              uint64_t slice_bytes);
/* Both digests of (file, offset, size) parts, each slice read once (pread into pinned
 * staging) and crossing PCIe once: s3h_sha256_file_parts for uploads that also send
 * Content-MD5.  Same arguments and errors as s3h_sha256_file_parts. */
/* Content-MD5 of (file, offset, size) parts, as s3h_sha256_file_parts. */
int s3h_md5_file_parts(const char *path, const uint64_t *offsets, const uint64_t *lengths,
                       uint64_t n, uint32_t *digests, int ndevices, uint64_t slice_bytes);
int s3h_sha256_md5_file_parts(const char *path, const uint64_t *offsets, const uint64_t *lengths,
                              uint64_t n, uint32_t *sha256_digests, uint32_t *md5_digests,
                              int ndevices, uint64_t slice_bytes);
int s3h_sha256_md5_batch_device(int device, const void *d_base, const uint64_t *offsets,
                                const uint64_t *lengths, uint64_t n, uint32_t *d_sha256,
                                uint32_t *d_md5, void *stream);

/* ---------------------------------------------------------------- size-aware routing
 * One part's chain runs at ~69 MB/s on the GPU and ~2.5 GB/s on one SHA-NI core, so a batch
 * of a few large parts -- the per-job batches of lib/src/upload.cpp:89-110, 136-140 -- is
 * faster on the CPU drop-in, and a batch of hundreds is faster on the GPU.  The routed entry
 * points take a route: S3H_ROUTE_GPU = the batched host path unchanged (the default
 * everywhere); S3H_ROUTE_CPU = the lib/hash drop-in (sha256::sha256, md5::md5, both digests in
 * one pass over each part) on s3h_host_threads' CPU count, parts longest first; S3H_ROUTE_AUTO
 * = whichever the model below estimates to finish first; S3H_ROUTE_SPLIT = both at once: the
 * CPU drop-in hashes the m longest parts on its threads while the GPU host path hashes the rest
 * (m from the model; a single part goes to the GPU; for pageable parts and file ranges the host
 * threads are divided between the GPU side's staging and the CPU side).  AUTO also splits when
 * the split is estimated at least 5 % faster than the better single route.  AUTO needs a
 * visible GPU (S3H_ENODEV otherwise): it chooses between paths with identical digests and is
 * never a fallback for a missing device.  *taken (if non-null) receives the route that ran.
 *   gpu_s = call_s + max(longest part / chain rate, bytes per device / feed rate)
 *           feed = h2d (pinned parts), min(h2d, staged memcpy) (pageable parts) or
 *                  min(h2d, staged pread) (file ranges)
 *   cpu_s = (longest-first schedule of the parts on k = min(n, threads) threads) / (rate(k) / k)
 *           rate(k) = min(k x one-thread rate, all-threads rate)
 * each for the digest set the call computes (SHA-256, MD5, or both), times the observed /
 * predicted ratio of earlier routed calls (the model is measured lazily per digest set and per
 * device, re-measured when a call diverges from its prediction by more than 25 % and every
 * s3h_route_refresh_calls calls). */
enum s3h_route { S3H_ROUTE_GPU = 0, S3H_ROUTE_CPU = 1, S3H_ROUTE_AUTO = 2, S3H_ROUTE_SPLIT = 3 };
/* Digest sets of the routing model: rate arrays are indexed by (set - 1). */
enum s3h_digests { S3H_DIGESTS_SHA256 = 1, S3H_DIGESTS_MD5 = 2, S3H_DIGESTS_BOTH = 3 };
/* The SHA-256 model (layout frozen at API version 1 + round 5's two trailing doubles). */
typedef struct {
  double cpu_bytes_per_s;   /* one host thread on the lib/hash drop-in (s3h_cpu_backend) */
  double chain_bytes_per_s; /* one part's chain on the GPU (the slowest visible device) */
  double h2d_bytes_per_s;   /* pinned host -> device copy (the slowest visible device) */
  double call_s;            /* fixed cost of one host-path GPU call (setup, launch, sync) */
  int cpu_threads;          /* host threads of the CPU route (affinity and cgroup quota) */
  int devices;              /* visible HIP devices */
  double cpu_all_bytes_per_s; /* all cpu_threads threads at once, aggregate: the CPU route on k
                               * threads runs at min(k x cpu_bytes_per_s, this) -- not linear
                               * (memory bandwidth, SMT siblings, the cgroup quota) */
  double staged_bytes_per_s;  /* pageable sources: cpu_threads threads' memcpy into pinned
                               * staging, aggregate; the GPU route is fed at min(h2d, this) */
} s3h_route_model_t;
/* The measured model (measures it on first use).  S3H_ENODEV without a GPU (cpu fields set). */
int s3h_route_model(s3h_route_model_t *m);
/* AUTO's choice for `lengths` under model *m (any model, e.g. a recorded one; pure host
 * arithmetic): returns S3H_ROUTE_GPU or S3H_ROUTE_CPU and both time estimates in seconds. */
int s3h_route_estimate(const s3h_route_model_t *m, const uint64_t *lengths, uint64_t n,
                       int ndevices, double *gpu_s, double *cpu_s);
/* The same for parts of a given source: S3H_SOURCE_PINNED (as s3h_route_estimate),
 * S3H_SOURCE_PAGEABLE (staged through pinned memory) or S3H_SOURCE_FILE (file ranges). */
enum s3h_source { S3H_SOURCE_PINNED = 0, S3H_SOURCE_PAGEABLE = 1, S3H_SOURCE_FILE = 2 };
int s3h_route_estimate_ex(const s3h_route_model_t *m, const uint64_t *lengths, uint64_t n,
                          int ndevices, int source, double *gpu_s, double *cpu_s);
/* The split route's plan under model *m (pure host arithmetic): with the parts ordered by length
 * (descending, ties by index), the first *cpu_parts go to the CPU and the rest to the GPU, and
 *   split_s(m) = max(gpu_s(the n - m shorter parts), cpu_s(the m longest)),  m = 1 .. n-1
 * (gpu_s / cpu_s as above on each side's parts); of the m with split_s(m) within 0.5 % of the
 * minimum (the GPU side's longest chain makes ranges of m tie), *cpu_parts = the one with the
 * smallest max(GPU side's bytes / devices / feed, cpu_s(m)), and *split_s = split_s(it)
 * (*cpu_parts = 0 when n == 1).  Pinned parts: the CPU side gets all cpu_threads threads
 * (*stage_threads = 0).  Pageable parts / file ranges: each GPU shard stages with
 * *stage_threads = tg threads, fed at min(H2D, staged rate x tg / threads), and the CPU side
 * gets the rest at the all-threads rate per thread; tg is the best of (threads / devices) x
 * {1, 4, 6, 8, 9} / 12 (env S3H_SPLIT_STAGE_THREADS fixes it). */
int s3h_route_split_estimate(const s3h_route_model_t *m, const uint64_t *lengths, uint64_t n,
                             int ndevices, int source, uint64_t *cpu_parts, int *stage_threads,
                             double *split_s);
/* The whole model, every digest set, with the observed corrections.  The caller sets `size`
 * (sizeof(s3h_route_rates_t) as it was compiled); the library writes at most that many bytes,
 * so a caller built against an older, shorter struct keeps working. */
typedef struct {
  uint32_t size;                  /* in: the struct size the caller knows; out: bytes written */
  uint32_t version;               /* out: the library's S3H_API_VERSION */
  int cpu_threads;                /* host threads of the CPU route */
  int devices;                    /* visible HIP devices */
  double cpu_bytes_per_s[3];      /* one host thread, per digest set (index = set - 1) */
  double cpu_all_bytes_per_s[3];  /* all cpu_threads threads, aggregate */
  double chain_bytes_per_s[3];    /* one GPU chain (the slowest device); [2]: both digests from one grid */
  double h2d_bytes_per_s;         /* pinned host -> device (the slowest device) */
  double staged_bytes_per_s;      /* staging memcpy of all cpu_threads threads */
  double call_s;                  /* fixed cost of one host-path GPU call */
  double gpu_factor[3];           /* observed / predicted wall time of routed calls, per digest */
  double cpu_factor[3];           /* set (EWMA; 1: none; 0 = 1 in s3h_route_choose) */
  uint64_t measurements;          /* times the model was (re)measured */
  uint64_t routed_calls;          /* AUTO / SPLIT calls observed */
  uint64_t divergences;           /* calls that differed from their prediction by > 25 % */
  double age_s;                   /* seconds since the last measurement */
  double staged_file_bytes_per_s; /* file ranges: cpu_threads threads' pread from the page cache
                                   * (0: price them at staged_bytes_per_s) */
} s3h_route_rates_t;
int s3h_route_rates(s3h_route_rates_t *r);
/* AUTO's decision for digest set `digests` under rates *r (pure host arithmetic; reads at most
 * r->size bytes, missing fields = 0, factors 0 = 1; the digest set's own factors apply). */
typedef struct {
  int route;           /* S3H_ROUTE_GPU, _CPU or _SPLIT */
  int stage_threads;   /* split: staging threads per GPU shard (0: pinned parts / no split) */
  uint64_t cpu_parts;  /* split: the longest parts on the CPU (0: no split plan) */
  double gpu_s, cpu_s; /* estimates with the observed factors */
  double split_s;      /* the split plan's estimate (0: none) */
} s3h_route_choice_t;
int s3h_route_choose(const s3h_route_rates_t *r, int digests, const uint64_t *lengths, uint64_t n,
                     int ndevices, int source, s3h_route_choice_t *out);
/* One device's lone-chain rate for a digest set and its pinned H2D rate (measured on first use). */
int s3h_route_device_rates(int device, int digests, double *chain_bytes_per_s,
                           double *h2d_bytes_per_s);
/* Re-measure the model after this many AUTO / SPLIT calls (default 64, env
 * S3H_ROUTE_REFRESH_CALLS; 0: only on divergence).  *previous (if non-null) gets the old value. */
int s3h_route_refresh_calls(int calls, int *previous);
/* Measurement / test hook: multiply one measured rate by `factor` until the model is next
 * measured -- a model taken while the GPU or the host was busy (tests/test_gpu_route_adapt.py). */
enum s3h_rate { S3H_RATE_CHAIN = 0, S3H_RATE_H2D = 1, S3H_RATE_CPU = 2, S3H_RATE_STAGED = 3 };
int s3h_route_scale(int which, double factor);
int s3h_sha256_batch_routed(const uint8_t *const *parts, const uint64_t *lengths, uint64_t n,
                            uint32_t *digests, int ndevices, int route, int *taken);
int s3h_sha256_file_parts_routed(const char *path, const uint64_t *offsets,
                                 const uint64_t *lengths, uint64_t n, uint32_t *digests,
                                 int ndevices, int route, int *taken);
/* Content-MD5 of host parts on a route (the CPU side: md5::md5). */
int s3h_md5_batch_routed(const uint8_t *const *parts, const uint64_t *lengths, uint64_t n,
                         uint32_t *digests, int ndevices, int route, int *taken);
/* Both upload headers on a route: the GPU side is s3h_sha256_md5_batch_host /
 * _file_parts (one grid, one PCIe pass), the CPU side hashes each part with SHA-256 and MD5 in
 * one pass over memory (64 KiB chunks while they sit in cache); the model prices both digests
 * (a CPU MD5 runs at ~1.0 GB/s per thread, both digests at ~0.7: the dual CPU route is ~3.5x
 * slower per thread than SHA-256 alone, so the GPU wins at far fewer parts). */
int s3h_sha256_md5_batch_routed(const uint8_t *const *parts, const uint64_t *lengths, uint64_t n,
                                uint32_t *sha256_digests, uint32_t *md5_digests, int ndevices,
                                int route, int *taken);
int s3h_sha256_md5_file_parts_routed(const char *path, const uint64_t *offsets,
                                     const uint64_t *lengths, uint64_t n, uint32_t *sha256_digests,
                                     uint32_t *md5_digests, int ndevices, int route, int *taken);

/* ---------------------------------------------------------------- verification
 * Download-side check of parts against known digests (ranged GETs of
 * lib/src/download.cpp:88-103; expected = the uploader's x-amz-content-sha256 / Content-MD5).
 * mismatch[i] = 1 when part i differs; *mismatches = their count.  Blocking.
 * Device form: d_expected (n x words) and d_mismatch (n bytes) are device pointers. */
int s3h_verify_batch_device(int device, int algo, const void *d_base, const uint64_t *offsets,
                            const uint64_t *lengths, uint64_t n, const uint32_t *d_expected,
                            uint8_t *d_mismatch, uint64_t *mismatches, void *stream);
int s3h_verify_batch_host(int algo, const uint8_t *const *parts, const uint64_t *lengths,
                          uint64_t n, const uint32_t *expected, uint8_t *mismatch,
                          uint64_t *mismatches, int ndevices);
/* The host form on a route (size-aware routing above): S3H_ROUTE_GPU = s3h_verify_batch_host;
 * CPU / SPLIT / AUTO hash as s3h_sha256_batch_routed / s3h_md5_batch_routed do (either
 * algorithm, priced by its own rates), then compare.  *taken (if non-null) receives the route
 * that ran. */
int s3h_verify_batch_routed(int algo, const uint8_t *const *parts, const uint64_t *lengths,
                            uint64_t n, const uint32_t *expected, uint8_t *mismatch,
                            uint64_t *mismatches, int ndevices, int route, int *taken);

/* ---------------------------------------------------------------- multi-object streams
 * n messages (objects) hashed incrementally as their bytes arrive in chunks: the batched,
 * device-resident form of lib/hash's chunked API -- sha256_stream (sha256.cpp:84-144) for the
 * appends, and the DOCUMENTED contract of sha256_next (sha256.h:73-89: chunks of one buffer,
 * the last one padded with the buffer's TOTAL length) for the finish.  (The reference's
 * sha256_next pads with the chunk length and hashes unpadded data)
 *   update: appends chunk i (lengths[i] bytes, any alignment, 0 allowed) to message i.
 *           Whole 64-B blocks are compressed on the GPU; each message's < 64-B remainder is
 *           carried on the device into the next update.  Asynchronous on `stream`; the host
 *           arrays may be reused on return, the device chunks must stay valid until the
 *           stream reaches this point.  An object's calls run on the device in call order,
 *           whichever stream each is given (each waits for the previous call's work).
 *   final:  pads every message with its total length, writes n digests (words as in the
 *           batch API) and resets the object to n empty messages.
 * The chaining state, carries and total lengths live on the device (n x 104 B); one object
 * may be driven from one host thread at a time.  MD5 (algo 1) follows md5_stream/md5_file. */
typedef struct s3h_stream_s *s3h_stream_t;
int s3h_stream_create(int device, int algo, uint64_t n, int kernel, s3h_stream_t *out);
int s3h_stream_update_device(s3h_stream_t s, const void *d_base, const uint64_t *offsets,
                             const uint64_t *lengths, void *stream);
int s3h_stream_final_device(s3h_stream_t s, uint32_t *d_digests, void *stream);
/* Host-memory forms: chunks[i] may be null when lengths[i] == 0.  update_host returns once
 * the chunks have been copied out of the caller's memory (they may be reused on return); its
 * hash runs on the device while the caller prepares the next update, whose copy overlaps it.
 * Page-locked chunks are DMA'd directly; pageable ones go through pinned pieces filled by copy
 * threads on the device's NUMA node.  final_host waits for every update and checks the
 * launches' device error words like s3h_plan_status (a fault of any update fails it). */
int s3h_stream_update_host(s3h_stream_t s, const uint8_t *const *chunks, const uint64_t *lengths);
int s3h_stream_final_host(s3h_stream_t s, uint32_t *digests);
/* Device forms: waits for `stream` and reports (and clears) a fault of any update / final
 * launch since the last check, as s3h_plan_status does for a plan. */
int s3h_stream_status(s3h_stream_t s, void *stream);
/* Update launches that found their plan's device slots in place (equal chunk lengths at
 * offsets moved by one constant: the base pointer moves, no re-sort, no copies) and those
 * that re-sorted and uploaded the slots.  Host counters, no device sync.  A call that fails
 * after queueing work leaves the object failed: later calls return S3H_EINVAL (destroy it). */
int s3h_stream_stats(s3h_stream_t s, uint64_t *slot_reuses, uint64_t *slot_refills);
/* Bytes appended so far to message i (host bookkeeping; no device sync). */
int s3h_stream_total(s3h_stream_t s, uint64_t i, uint64_t *total);
int s3h_stream_destroy(s3h_stream_t s);

/* ---------------------------------------------------------------- synthetic inputs
 * Fill part i (at d_base + offsets[i], 8-B aligned, lengths[i] bytes) with generator
 * G(seed, part_ids[i], lengths[i]) of SURVEY.md 8(d).  Asynchronous on `stream`. */
int s3h_generate_parts(int device, void *d_base, const uint64_t *offsets,
                       const uint64_t *lengths, const uint64_t *part_ids, uint64_t n,
                       uint64_t seed, void *stream);

/* ---------------------------------------------------------------- CPU drop-in (C view)
 * C entry points of the lib/hash drop-in that the same library exports in C++ form
 * (namespace sha256, include/sha256.h).  Single messages: CPU, never the GPU. */
void s3h_cpu_sha256(const uint8_t *data, uint64_t length, uint32_t hash[8]);
void s3h_cpu_hmac256(const uint8_t *data, uint64_t length, const uint8_t *key,
                     uint64_t key_length, uint8_t mac[32]);
/* MD5 drop-in (md5::md5, include/md5.h): hash[0..3], digest bytes = words in LE order. */
void s3h_cpu_md5(const uint8_t *data, uint64_t length, uint32_t hash[4]);
/* S3 multipart ETag of an object from its parts' MD5 digests (n x 4 words, as the MD5 batch
 * entry points return them, in part order): lowercase hex of MD5(the n 16-byte digests
 * concatenated) + "-" + n, NUL-terminated, into out (out_len >= S3H_ETAG_MAX).  This is the
 * ETag CompleteMultipartUpload returns (lib/src/api/multipart_upload.cpp:162-183); an
 * uploader compares it with the server's.  CPU (16 B per part).  S3H_EINVAL for n == 0. */
#define S3H_ETAG_MAX 56
int s3h_multipart_etag(const uint32_t *md5_digests, uint64_t n, char *out, uint64_t out_len);
/* lowercase hex of the 32 digest bytes + NUL (sha256::hash_to_text). */
void s3h_hash_to_text(const uint32_t hash[8], char text[65]);
/* "sha-ni" or "scalar": which compression the CPU drop-in dispatched to. */
const char *s3h_cpu_backend(void);

#ifdef __cplusplus
}
#endif
#endif /* S3HASH_H */
