// Flat C API of libstereo_amd.so (engine lifecycle + per-frame execution).  Kernel-level
// entry points are declared in sa/kernels.h.
#pragma once
#ifdef __cplusplus
extern "C" {
#endif

#define SA_VERSION_STRING "stereoalgorithms_amd 0.1.0 (gfx950)"

const char* sa_version(void);
const char* sa_last_error(void);
void* sa_engine_create(const char* model, const char* weights, int height, int width, int batch,
                       int iters, int device, int use_graph, unsigned long long seed);
void sa_engine_destroy(void* engine);
int sa_engine_set_q(void* engine, const float* q16);
int sa_engine_set_rectify_maps(void* engine, const float* map_left, const float* map_right);
int sa_engine_run_device(void* engine, const void* left, const void* right, float* disp,
                         float* cloud, int rectify, void* stream, void* rect_left, void* rect_right);
// Host buffers in / out.  A caller buffer passed for the same role (left, right, disp, cloud) on two consecutive
// frames is mapped into the GPU (hipHostRegister) and read / written by the frame graph over PCIe; it stays mapped
// until a different buffer is passed for that role or the engine is destroyed, so it must not be freed (or
// reallocated at the same address) before then.  Transient buffers: use sa_engine_host_buffers' staging instead,
// or SA_HOST_REGISTER=0 (copies through the pinned staging).
int sa_engine_run_host(void* engine, void* left, void* right, float* disp, float* cloud,
                       int rectify);
long long sa_engine_device_bytes(void* engine);
// run_host's pinned staging (pass these pointers back to run_host to skip the host-side copies) and the timing
// split of the last run_host (ms: total, input copies, enqueue, wait + output copies[, H2D, graph, D2H]; H2D is -1
// when the frame graph read the images itself over PCIe -- zero-copy inputs -- and 'graph' includes that read)
void sa_engine_host_buffers(void* engine, void** left, void** right, float** disp, float** cloud);
int sa_engine_host_times(void* engine, float* out, int max);
const float* sa_engine_aux_output(void* engine, int* n);
void* sa_engine_stream(void* engine);
// tuned-plan cache: the engine's plan file ("" = none), the conv shapes it had to time at build,
// the process-wide count of timed shapes, and a reset of the in-process plan (tests)
const char* sa_engine_plan_path(void* engine);
const char* sa_engine_tactics_digest(void* engine);        // 16-hex digest of the tactics the engine launches
int sa_engine_plan_export(void* engine, const char* file);  // its plan entries as a plan file; 0 or errno
void sa_conv_plan_pin(int on);                             // later plan-file loads keep existing entries
long sa_engine_tuned_shapes(void* engine);
long sa_engine_nonzero_splitk_counters(void* engine);
long sa_conv_tune_count(void);
long sa_conv_tune_rejects(void);
void sa_conv_plan_clear(void);
void sa_conv_plan_put(const char* key, int cfg, int splitk, float us);
int sa_conv_plan_save(const char* file, const char* keys);  // keys newline-separated; 0 or errno
int sa_conv_plan_load(const char* file);                    // entries in the file, -1 absent, -2 another build / no header
void sa_conv_plan_cache_append(const char* key, int cfg, int splitk, float us);  // SA_PLAN_CACHE append
long sa_conv_plan_entries(void);
// per-stage device times of the last frame (SA_STAGE_TIMES=1): returns the count (<= max), fills
// ms[i] and names[i] (pointers valid for the engine's lifetime)
int sa_engine_stage_times(void* engine, float* ms, const char** names, int max);

// The per-model facade (sa::StereoAlgorithm, sa/algorithm.h): calibration YAML, rectification maps and the
// reference's Run semantics.  create returns NULL on failure (message: sa_last_error).  run takes contiguous BGR
// u8 [rows][cols][3] images (rectified in place when `rectify`), writes disparity [rows][cols] fp32 and, when
// `cloud` is not NULL, the point cloud [rows][cols][6].
void* sa_algorithm_create(const char* model, int gpu_id, const char* calibration_path, const char* default_preset);
int sa_algorithm_run(void* alg, unsigned char* left, unsigned char* right, int rows, int cols, float* disparity,
                     float* cloud, int rectify);
int sa_algorithm_frame_size(void* alg, int* rows, int* cols);
float sa_algorithm_last_ms(void* alg);
void sa_algorithm_destroy(void* alg);

#ifdef __cplusplus
}
#endif
