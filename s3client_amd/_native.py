"""ctypes binding of libs3hash.so (the C-ABI declared in include/s3hash.h).

The library is built in-tree (``make`` at the repo root, or ``__graft_entry__.build()``) to
``s3client_amd/lib/libs3hash.so``.  There is no fallback: if the library is missing, every
entry point raises, and the batched GPU entry points raise when no HIP device is visible.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libs3hash.so")
# Kernel experiments only (`make exp` builds variants under tools/exp/): S3H_LIBRARY points the
# Python layer at one of them.  Unset in every test, smoke and default bench run.
LIB_PATH = os.environ.get("S3H_LIBRARY", LIB_PATH)

S3H_OK, S3H_EINVAL, S3H_ENODEV, S3H_EHIP, S3H_ENOMEM = 0, -1, -2, -3, -4
KERNEL_AUTO, KERNEL_LANE, KERNEL_PC, KERNEL_PAIR, KERNEL_QUAD, KERNEL_SKEW, KERNEL_SKEWP = 0, 1, 2, 3, 4, 5, 6
KERNEL_SKEWS = 7
KERNEL_NAMES = {KERNEL_AUTO: "auto", KERNEL_LANE: "lane", KERNEL_PC: "pc", KERNEL_PAIR: "pair",
                KERNEL_QUAD: "quad", KERNEL_SKEW: "skew", KERNEL_SKEWP: "skewp", KERNEL_SKEWS: "skews"}
KERNEL_IDS = {v: k for k, v in KERNEL_NAMES.items()}

# every symbol include/s3hash.h declares (tests check the library exports all of them)
C_ABI_SYMBOLS = (
    "s3h_last_error", "s3h_api_version", "s3h_device_count",
    "s3h_plan_create", "s3h_plan_destroy", "s3h_plan_launch", "s3h_plan_launch_range",
    "s3h_plan_info", "s3h_sha256_batch_device", "s3h_sha256_batch_host",
    "s3h_generate_parts", "s3h_cpu_sha256", "s3h_cpu_hmac256", "s3h_hash_to_text",
    "s3h_cpu_backend", "s3h_cpu_md5", "s3h_plan_create_ex", "s3h_plan_algo",
    "s3h_md5_batch_device", "s3h_md5_batch_host", "s3h_verify_batch_device",
    "s3h_verify_batch_host", "s3h_stream_create", "s3h_stream_update_device",
    "s3h_stream_final_device", "s3h_stream_update_host", "s3h_stream_final_host",
    "s3h_stream_total", "s3h_stream_destroy", "s3h_plan_set_clock_probe",
    "s3h_sha256_md5_batch_host", "s3h_sha256_md5_batch_device", "s3h_trim",
    "s3h_sha256_file_parts", "s3h_sha256_batch_host_on", "s3h_plan_groups",
    "s3h_sha256_md5_file_parts", "s3h_plan_status", "s3h_stream_status", "s3h_host_threads",
    "s3h_plan_dual_solo", "s3h_device_pci_bus_id", "s3h_multipart_etag",
    "s3h_route_model", "s3h_route_estimate", "s3h_sha256_batch_routed",
    "s3h_sha256_file_parts_routed", "s3h_pci_numa", "s3h_device_numa_node", "s3h_host_numa",
    "s3h_host_numa_info", "s3h_host_alloc", "s3h_host_free", "s3h_mem_node",
    "s3h_route_estimate_ex", "s3h_kernel_policy", "s3h_stream_stats", "s3h_plan_dual_layout",
    "s3h_dual_layout", "s3h_route_split_estimate", "s3h_verify_batch_routed",
    # round 6: digest-set routing, adaptive model, host thread plan, strict pinned allocation
    "s3h_route_rates", "s3h_route_choose", "s3h_route_device_rates", "s3h_route_refresh_calls",
    "s3h_route_scale", "s3h_md5_batch_routed", "s3h_sha256_md5_batch_routed",
    "s3h_sha256_md5_file_parts_routed", "s3h_md5_file_parts", "s3h_host_plan",
    "s3h_host_alloc_ex", "s3h_device_power_cap", "s3h_pci_power_cap",
)
POLICY_IDS = {"throughput": 0, "efficiency": 1, "power": 2}
POLICY_NAMES = {v: k for k, v in POLICY_IDS.items()}
SOURCE_IDS = {"pinned": 0, "pageable": 1, "file": 2}
NUMA_LOCAL, NUMA_OFF = -1, -2
ROUTE_GPU, ROUTE_CPU, ROUTE_AUTO, ROUTE_SPLIT = 0, 1, 2, 3
ROUTE_IDS = {"gpu": ROUTE_GPU, "cpu": ROUTE_CPU, "auto": ROUTE_AUTO, "split": ROUTE_SPLIT}
ROUTE_NAMES = {v: k for k, v in ROUTE_IDS.items()}


class RouteModel(ctypes.Structure):
    """s3h_route_model_t (include/s3hash.h)."""
    _fields_ = [("cpu_bytes_per_s", ctypes.c_double), ("chain_bytes_per_s", ctypes.c_double),
                ("h2d_bytes_per_s", ctypes.c_double), ("call_s", ctypes.c_double),
                ("cpu_threads", ctypes.c_int), ("devices", ctypes.c_int),
                ("cpu_all_bytes_per_s", ctypes.c_double), ("staged_bytes_per_s", ctypes.c_double)]


DIGESTS_SHA256, DIGESTS_MD5, DIGESTS_BOTH = 1, 2, 3
DIGESTS_IDS = {"sha256": DIGESTS_SHA256, "md5": DIGESTS_MD5, "both": DIGESTS_BOTH}
RATE_IDS = {"chain": 0, "h2d": 1, "cpu": 2, "staged": 3}
HOST_ALLOC_STRICT = 1


class RouteRates(ctypes.Structure):
    """s3h_route_rates_t (include/s3hash.h): size-carrying, every digest set."""
    _fields_ = [("size", ctypes.c_uint32), ("version", ctypes.c_uint32),
                ("cpu_threads", ctypes.c_int), ("devices", ctypes.c_int),
                ("cpu_bytes_per_s", ctypes.c_double * 3),
                ("cpu_all_bytes_per_s", ctypes.c_double * 3),
                ("chain_bytes_per_s", ctypes.c_double * 3),
                ("h2d_bytes_per_s", ctypes.c_double), ("staged_bytes_per_s", ctypes.c_double),
                ("call_s", ctypes.c_double), ("gpu_factor", ctypes.c_double * 3),
                ("cpu_factor", ctypes.c_double * 3), ("measurements", ctypes.c_uint64),
                ("routed_calls", ctypes.c_uint64), ("divergences", ctypes.c_uint64),
                ("age_s", ctypes.c_double), ("staged_file_bytes_per_s", ctypes.c_double)]


class RouteChoice(ctypes.Structure):
    """s3h_route_choice_t (include/s3hash.h)."""
    _fields_ = [("route", ctypes.c_int), ("stage_threads", ctypes.c_int),
                ("cpu_parts", ctypes.c_uint64), ("gpu_s", ctypes.c_double),
                ("cpu_s", ctypes.c_double), ("split_s", ctypes.c_double)]


class HostPlan(ctypes.Structure):
    """s3h_host_plan_t (include/s3hash.h)."""
    _fields_ = [("cpus", ctypes.c_int), ("affinity_cpus", ctypes.c_int),
                ("cpu_quota", ctypes.c_double), ("devices", ctypes.c_int),
                ("staging_threads_per_device", ctypes.c_int), ("threads", ctypes.c_int),
                ("oversubscribed", ctypes.c_int), ("below_saturation", ctypes.c_int),
                ("node_oversubscribed", ctypes.c_int), ("split_cpu_threads_pinned", ctypes.c_int),
                ("split_candidates", ctypes.c_int), ("split_stage_min", ctypes.c_int),
                ("split_stage_max", ctypes.c_int), ("split_cpu_threads_min", ctypes.c_int),
                ("split_cpu_threads_max", ctypes.c_int)]


class HostPlanDevice(ctypes.Structure):
    """s3h_host_plan_device_t (include/s3hash.h)."""
    _fields_ = [("node", ctypes.c_int), ("bind_node", ctypes.c_int), ("bind_cpus", ctypes.c_int),
                ("bind_first_cpu", ctypes.c_int), ("bind_last_cpu", ctypes.c_int),
                ("staging_threads", ctypes.c_int)]


class HostNuma(ctypes.Structure):
    """s3h_host_numa_t (include/s3hash.h)."""
    _fields_ = [("device_node", ctypes.c_int), ("target_node", ctypes.c_int),
                ("bound_cpus", ctypes.c_int), ("staging_node", ctypes.c_int),
                ("threads_node", ctypes.c_int), ("copy_threads", ctypes.c_int)]


ALGO_SHA256, ALGO_MD5 = 0, 1
ALGO_IDS = {"sha256": ALGO_SHA256, "md5": ALGO_MD5}
DIGEST_WORDS = {ALGO_SHA256: 8, ALGO_MD5: 4}
# the lib/hash drop-in (C++ mangled names identical to the reference's libs3client.a)
CXX_DROPIN_SYMBOLS = (
    "_ZN6sha2566sha256EPKhmPj",          # sha256::sha256(const uint8_t*, size_t, uint32_t*)
    "_ZN6sha25613sha256_streamEPjPKhm",  # sha256::sha256_stream(uint32_t*, const uint8_t*, uint64_t)
    "_ZN6sha25611sha256_nextEPKhjPjmPh", # sha256::sha256_next(...)
    "_ZN6sha25610print_hashEPj",         # sha256::print_hash(uint32_t*)
    "_ZN6sha25611sha256_fileEPKcPj",     # sha256::sha256_file(const char*, uint32_t*)
    "_Z7hmac256PKhmS0_mPh",              # hmac256(...)
    "_Z12alloc_paddedmmPmPh",            # alloc_padded(...)
    "_ZN3md510md5_streamEPjPKhm",        # md5::md5_stream(uint32_t*, const uint8_t*, uint64_t)
    "_ZN3md53md5EPKhmPj",                # md5::md5(const uint8_t*, size_t, uint32_t*)
    "_ZN3md510print_hashEPj",            # md5::print_hash(uint32_t*)
    "_ZN3md58md5_fileEPKcPj",            # md5::md5_file(const char*, uint32_t*)
)


class S3HashError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"s3hash error {code}: {msg}")
        self.code = code


_lib = None
_lock = threading.Lock()

u64p = ctypes.POINTER(ctypes.c_uint64)
u32p = ctypes.POINTER(ctypes.c_uint32)


def lib() -> ctypes.CDLL:
    """Load libs3hash.so once; raise loudly if it has not been built."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise S3HashError(S3H_EINVAL, f"{LIB_PATH} missing: run `make` (or "
                                  "__graft_entry__.build()) -- there is no fallback path")
            # One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64 and
            # libhsa-runtime64 (SONAME libamdhip64.so.7, like /opt/rocm's), but torch's own
            # libraries NEED the unversioned names: loaded AFTER this library, torch maps a
            # second HIP + ROCr instance and this library's runtime loses the device ("no HIP
            # device visible" on its first GPU call after torch.cuda.init(); tools/
            # cpu_route_context_probe.py on the box).  With torch loaded first this library's
            # NEEDED libamdhip64.so.7 resolves to torch's runtime by SONAME.
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            L = ctypes.CDLL(LIB_PATH)
            L.s3h_last_error.restype = ctypes.c_char_p
            L.s3h_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
            L.s3h_device_pci_bus_id.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
            L.s3h_pci_numa.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                       ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
            L.s3h_device_numa_node.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                               ctypes.c_char_p, ctypes.c_int]
            L.s3h_host_numa.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
            L.s3h_host_numa_info.argtypes = [ctypes.c_int, ctypes.POINTER(HostNuma)]
            L.s3h_host_alloc.argtypes = [ctypes.c_int, ctypes.c_uint64,
                                         ctypes.POINTER(ctypes.c_void_p)]
            L.s3h_host_free.argtypes = [ctypes.c_void_p]
            L.s3h_kernel_policy.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
            L.s3h_device_power_cap.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
            L.s3h_pci_power_cap.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double)]
            L.s3h_stream_stats.argtypes = [ctypes.c_void_p, u64p, u64p]
            L.s3h_plan_dual_layout.argtypes = [ctypes.c_void_p, u32p, ctypes.POINTER(ctypes.c_int)]
            L.s3h_dual_layout.argtypes = [u64p, ctypes.c_uint64, ctypes.c_int, u32p,
                                          ctypes.POINTER(ctypes.c_int)]
            L.s3h_mem_node.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
            L.s3h_plan_create.argtypes = [ctypes.c_int, u64p, u64p, ctypes.c_uint64, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_void_p)]
            L.s3h_plan_create_ex.argtypes = [ctypes.c_int, ctypes.c_int, u64p, u64p,
                                             ctypes.c_uint64, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_void_p)]
            L.s3h_plan_algo.argtypes = [ctypes.c_void_p]
            L.s3h_plan_destroy.argtypes = [ctypes.c_void_p]
            L.s3h_plan_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p]
            L.s3h_plan_launch_range.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                ctypes.c_void_p]
            L.s3h_plan_status.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            L.s3h_stream_status.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            L.s3h_host_threads.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
            L.s3h_plan_set_clock_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                                   ctypes.POINTER(ctypes.c_uint32)]
            L.s3h_plan_info.argtypes = [ctypes.c_void_p, u64p, u64p, u64p,
                                        ctypes.POINTER(ctypes.c_int), u32p]
            L.s3h_plan_groups.argtypes = [ctypes.c_void_p, u32p, u32p]
            L.s3h_plan_dual_solo.argtypes = [ctypes.c_void_p, u32p]
            L.s3h_sha256_batch_device.argtypes = [ctypes.c_int, ctypes.c_void_p, u64p, u64p,
                                                  ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
            for name in ("s3h_sha256_batch_host", "s3h_md5_batch_host"):
                getattr(L, name).argtypes = [ctypes.POINTER(ctypes.c_void_p), u64p,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                                             ctypes.c_uint64]
            L.s3h_sha256_batch_host_on.argtypes = [ctypes.POINTER(ctypes.c_void_p), u64p,
                                                   ctypes.c_uint64, ctypes.c_void_p,
                                                   ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                                   ctypes.c_uint64]
            L.s3h_sha256_file_parts.argtypes = [ctypes.c_char_p, u64p, u64p, ctypes.c_uint64,
                                                ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64]
            L.s3h_sha256_md5_file_parts.argtypes = [ctypes.c_char_p, u64p, u64p, ctypes.c_uint64,
                                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                    ctypes.c_uint64]
            L.s3h_sha256_md5_batch_host.argtypes = [ctypes.POINTER(ctypes.c_void_p), u64p,
                                                    ctypes.c_uint64, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_int,
                                                    ctypes.c_uint64]
            L.s3h_sha256_md5_batch_device.argtypes = [ctypes.c_int, ctypes.c_void_p, u64p, u64p,
                                                      ctypes.c_uint64, ctypes.c_void_p,
                                                      ctypes.c_void_p, ctypes.c_void_p]
            L.s3h_verify_batch_host.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), u64p,
                                                ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                                u64p, ctypes.c_int]
            L.s3h_verify_batch_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, u64p,
                                                  u64p, ctypes.c_uint64, ctypes.c_void_p,
                                                  ctypes.c_void_p, u64p, ctypes.c_void_p]
            L.s3h_md5_batch_device.argtypes = [ctypes.c_int, ctypes.c_void_p, u64p, u64p,
                                               ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
            L.s3h_generate_parts.argtypes = [ctypes.c_int, ctypes.c_void_p, u64p, u64p, u64p,
                                             ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
            L.s3h_cpu_sha256.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
            L.s3h_cpu_sha256.restype = None
            L.s3h_cpu_hmac256.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.c_uint64, ctypes.c_void_p]
            L.s3h_cpu_hmac256.restype = None
            L.s3h_hash_to_text.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
            L.s3h_hash_to_text.restype = None
            L.s3h_cpu_backend.restype = ctypes.c_char_p
            L.s3h_cpu_md5.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
            L.s3h_cpu_md5.restype = None
            L.s3h_route_model.argtypes = [ctypes.POINTER(RouteModel)]
            L.s3h_route_estimate.argtypes = [ctypes.POINTER(RouteModel), u64p, ctypes.c_uint64,
                                             ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_double)]
            L.s3h_route_estimate_ex.argtypes = [ctypes.POINTER(RouteModel), u64p, ctypes.c_uint64,
                                                ctypes.c_int, ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_double),
                                                ctypes.POINTER(ctypes.c_double)]
            L.s3h_route_split_estimate.argtypes = [ctypes.POINTER(RouteModel), u64p, ctypes.c_uint64,
                                                   ctypes.c_int, ctypes.c_int,
                                                   ctypes.POINTER(ctypes.c_uint64),
                                                   ctypes.POINTER(ctypes.c_int),
                                                   ctypes.POINTER(ctypes.c_double)]
            L.s3h_verify_batch_routed.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), u64p,
                                                  ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.POINTER(ctypes.c_uint64), ctypes.c_int,
                                                  ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
            L.s3h_sha256_batch_routed.argtypes = [ctypes.POINTER(ctypes.c_void_p), u64p,
                                                  ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                                                  ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
            L.s3h_sha256_file_parts_routed.argtypes = [ctypes.c_char_p, u64p, u64p,
                                                       ctypes.c_uint64, ctypes.c_void_p,
                                                       ctypes.c_int, ctypes.c_int,
                                                       ctypes.POINTER(ctypes.c_int)]
            L.s3h_route_rates.argtypes = [ctypes.POINTER(RouteRates)]
            L.s3h_route_choose.argtypes = [ctypes.POINTER(RouteRates), ctypes.c_int, u64p,
                                           ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(RouteChoice)]
            L.s3h_route_device_rates.argtypes = [ctypes.c_int, ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_double),
                                                 ctypes.POINTER(ctypes.c_double)]
            L.s3h_route_refresh_calls.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
            L.s3h_route_scale.argtypes = [ctypes.c_int, ctypes.c_double]
            L.s3h_md5_batch_routed.argtypes = L.s3h_sha256_batch_routed.argtypes
            L.s3h_sha256_md5_batch_routed.argtypes = [ctypes.POINTER(ctypes.c_void_p), u64p,
                                                      ctypes.c_uint64, ctypes.c_void_p,
                                                      ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                      ctypes.POINTER(ctypes.c_int)]
            L.s3h_sha256_md5_file_parts_routed.argtypes = [ctypes.c_char_p, u64p, u64p,
                                                           ctypes.c_uint64, ctypes.c_void_p,
                                                           ctypes.c_void_p, ctypes.c_int,
                                                           ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
            L.s3h_md5_file_parts.argtypes = L.s3h_sha256_file_parts.argtypes
            L.s3h_host_plan.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                        ctypes.c_char_p, ctypes.c_double,
                                        ctypes.POINTER(HostPlan), ctypes.POINTER(HostPlanDevice)]
            L.s3h_host_alloc_ex.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_void_p)]
            L.s3h_multipart_etag.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_char_p,
                                             ctypes.c_uint64]
            L.s3h_stream_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                            ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
            L.s3h_stream_update_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, u64p, u64p,
                                                   ctypes.c_void_p]
            L.s3h_stream_final_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p]
            L.s3h_stream_update_host.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                                 u64p]
            L.s3h_stream_final_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            L.s3h_stream_total.argtypes = [ctypes.c_void_p, ctypes.c_uint64, u64p]
            L.s3h_stream_destroy.argtypes = [ctypes.c_void_p]
            _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != S3H_OK:
        raise S3HashError(rc, lib().s3h_last_error().decode(errors="replace"))
