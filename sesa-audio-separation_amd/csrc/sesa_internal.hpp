// Internal launchers shared between translation units of libsesa.
#pragma once
#include <hip/hip_runtime.h>

namespace sesa {

int get_spectral_tables(const float2** tw4096, const float2** twN, const float** window);

// layout 0 = reference layout, 1 = MDX23C channels-last sub-band image (see sesa_spectral.hip).
int stft_launch(const float* x, int n_sig, int len, int hop, int dim_f, int layout, int nsub, float* out,
                hipStream_t st);
int istft_launch(const float* spec, int n_sig, int dim_f, int frames, int hop, int layout, int nsub, int ni,
                 float* out, float* frame_ws, hipStream_t st);

}  // namespace sesa

namespace sesa {
// launch timing hooks (sesa_profile.hip): token = profile_begin(st); <launch>; profile_end(token, ...)
bool profiling();
void* profile_begin(hipStream_t st);
// work: algorithmic FLOPs (compute classes) or bytes (streaming classes); bytes: the algorithmic HBM bytes of a
// compute-class launch (0: not stated)
void profile_end(void* token, hipStream_t st, int kclass, double work, double bytes = 0.0);
// checksum of a launch's output bytes into the host thread's trace buffer, if one is set (sesa_debug_trace_begin)
void debug_trace(hipStream_t st, int kclass, const void* p, size_t bytes);
// the byte range every later profile_end checksums while a trace is open (nullptr: none)
void debug_trace_range(const void* p, size_t bytes);
// SESA_DEBUG_ONLY: true for a launch of a class other than the selected one (the forward skips it)
bool debug_skip(int kclass);
}  // namespace sesa
