// Internal runtime helpers shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>

#include "orb_kernels.h"

struct orbx_ctx;

namespace orbpl {
int hip_fail(hipError_t e, const char* what, int line);
int arg_fail(const char* msg);
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device):
// HIP function attributes are per device, so a process-wide flag would skip
// the second device. Thread-safe; the current device is hipGetDevice's.
void set_smem_attr(const void* fn, size_t bytes);
// compute units of the current device (cached per device)
int device_cu_count();
// hardware queues the HIP runtime runs with, as recorded at library load
// (orbpl_runtime.cpp: not re-read from the environment)
int hw_queues();
extern int g_hw_queues, g_runtime_started, g_queues_set_by_lib;
// would a lines tracker of n_streams split its LSD batch (track_runtime.cpp)
bool lsd_split_decision(int n_streams);
// Run `init` once per (key, device) (thread-safe); returns true the first time.
bool once_per_device(const void* key);
int orbx_run(orbx_ctx* c, const uint8_t* d_imgs, int batch, int stride, long long frame_pitch,
             orbpl_keypoint_dev* d_kps, uint8_t* d_desc, int kp_pitch, int* d_n,
             hipEvent_t* ext_events = nullptr, hipEvent_t* ext_kernels = nullptr);
// ext_events[0..5]: start, pyramid done, (empty blur stage), FAST done,
// octree done, orientation + descriptors done (on the ctx stream; with the
// level pipeline 1..5 all mark the join of the FAST stream);
// ext_kernels[2 (K kFastGroups + g)], [.. + 1]: the FAST (K = 0), octree (1)
// and orientation + descriptor (2) launch of level group g bracketed on its
// stream, unused pairs recorded back to back: a stage's time is the sum of
// its pairs, its kernel time without the waits between groups
constexpr int kFastGroups = 4;
constexpr int kKernelBrackets = 6 * kFastGroups;
hipStream_t orbx_stream(orbx_ctx* c);
struct OrbGeom;
int orbx_device_pyramid(orbx_ctx* c, int frame, const uint8_t** base, const OrbGeom** geom,
                        hipStream_t* stream);
}  // namespace orbpl
