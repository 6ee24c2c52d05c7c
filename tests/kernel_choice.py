"""AUTO's kernel for 4,097 - 32 x CUs parts under the default "power" policy
(s3client_amd/csrc/plan.cpp resolve_kernel): skewp when the board's power cap is known and
below the 1,500 W the shared-SIMD skews kernel needs to hold its clock, skews otherwise."""
import s3client_amd as s3

SKEWS_FULL_CLOCK_W = 1500.0


def shared_range_kernel(device: int = 0) -> str:
    cap = s3.device_power_cap(device)
    return "skewp" if 0 < cap < SKEWS_FULL_CLOCK_W else "skews"
