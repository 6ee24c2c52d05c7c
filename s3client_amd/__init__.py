"""s3client_amd -- MI355X-native (gfx950) batched SHA-256 for S3 upload-part payload hashing.

Drop-in for uv-cpp/s3client's lib/hash on the payload-hashing path; see DESIGN.md.
"""
from .hashing import (Plan, device_count, digests_to_text, generate_parts, hash_to_text,
                      hmac256, nblocks, sha256, sha256_batch_device, sha256_batch_host,
                      cpu_backend, md5, md5_batch_device, md5_batch_host, multipart_etag,
                      verify_batch_device, verify_batch_host, verify_batch_routed, Stream,
                      sha256_md5_batch_device, sha256_md5_batch_host, sha256_file_parts,
                      sha256_md5_file_parts,
                      trim, sha256_batch_host_on, host_threads, device_pci_bus_id,
                      route_model, route_estimate, route_split_estimate, sha256_batch_routed,
                      sha256_file_parts_routed, BufferParts, pci_numa, device_numa,
                      host_numa, host_numa_info, mem_node, PinnedBuffer,
                      kernel_policy, dual_layout, md5_batch_routed, sha256_md5_batch_routed,
                      sha256_md5_file_parts_routed, md5_file_parts, route_rates, route_choose,
                      route_device_rates, route_refresh_calls, route_scale, host_plan,
                      device_power_cap, pci_power_cap)
from .upload import upload_parts_geometry, UploadPart
from ._native import S3HashError, LIB_PATH

__all__ = ["BufferParts", "Plan", "device_count", "digests_to_text", "generate_parts", "hash_to_text",
           "hmac256", "nblocks", "sha256", "sha256_batch_device", "sha256_batch_host",
           "cpu_backend", "md5", "md5_batch_device", "md5_batch_host", "multipart_etag",
           "verify_batch_device", "verify_batch_host", "verify_batch_routed", "Stream",
           "sha256_md5_batch_device", "sha256_md5_batch_host", "sha256_file_parts",
           "sha256_md5_file_parts", "trim", "sha256_batch_host_on", "host_threads",
           "device_pci_bus_id", "route_model", "route_estimate", "route_split_estimate", "sha256_batch_routed",
           "sha256_file_parts_routed", "pci_numa", "device_numa", "host_numa", "host_numa_info",
           "mem_node", "PinnedBuffer", "kernel_policy", "dual_layout", "md5_batch_routed",
           "sha256_md5_batch_routed", "sha256_md5_file_parts_routed", "md5_file_parts",
           "route_rates", "route_choose", "route_device_rates", "route_refresh_calls",
           "route_scale", "host_plan", "device_power_cap", "pci_power_cap",
           "upload_parts_geometry", "UploadPart", "S3HashError", "LIB_PATH"]
