// aipstack_amd -- internal helpers shared by the host runtime and the kernel launchers.
#ifndef AIPSTACK_AMD_CHKSUM_INTERNAL_H
#define AIPSTACK_AMD_CHKSUM_INTERNAL_H

#include <hip/hip_runtime.h>

namespace aipstack_amd {

// Records `e` as this thread's last HIP error and maps it to a status code.
int check_hip(hipError_t e);

// Compute units of the current device (cached per device id); <= 0 on failure.
int device_cu_count();

// Frames a wave of the Rx-verify / Tx-fill kernels keeps in flight (tunable "frames":
// 1, 2 or 4; default 2).
int tuning_frames_in_flight();

}  // namespace aipstack_amd

#endif
