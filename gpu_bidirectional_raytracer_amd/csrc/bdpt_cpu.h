// bdpt_cpu.h -- the host (CPU) backend behind the C-ABI (bdpt_create with BDPT_DEVICE_CPU).
// Internal interface between bdpt_host.cpp and bdpt_cpu.cpp; no HIP in either signature.
#ifndef BDPT_CPU_H
#define BDPT_CPU_H

#include <stdint.h>

#include "../../include/bdpt.h"

struct bdpt_cpu_ctx;

bdpt_cpu_ctx* bdpt_cpu_create(const bdpt_sphere* spheres, unsigned n, int W, int H, const uint32_t* mt_params);
void bdpt_cpu_destroy(bdpt_cpu_ctx* c);
void bdpt_cpu_set_scene(bdpt_cpu_ctx* c, const bdpt_sphere* spheres, unsigned n);
void bdpt_cpu_set_camera(bdpt_cpu_ctx* c, const bdpt_camera* cam);
void bdpt_cpu_reset_accum(bdpt_cpu_ctx* c);
void bdpt_cpu_set_shard(bdpt_cpu_ctx* c, int shard, int nshards, int band_rows);
int bdpt_cpu_threads(const bdpt_cpu_ctx* c);
void bdpt_cpu_generate_rand(bdpt_cpu_ctx* c, unsigned seed);
void bdpt_cpu_light_pass(bdpt_cpu_ctx* c, int current_sample);
void bdpt_cpu_path_passes(bdpt_cpu_ctx* c, const unsigned* sid, const int* vlp, int npass);
bool bdpt_cpu_rand_ready(const bdpt_cpu_ctx* c);
bool bdpt_cpu_camera_set(const bdpt_cpu_ctx* c);
void bdpt_cpu_read_radiance(const bdpt_cpu_ctx* c, bdpt_vec* colors, unsigned* counter);
void bdpt_cpu_read_pixels(const bdpt_cpu_ctx* c, unsigned char* rgba);
void bdpt_cpu_read_rand(const bdpt_cpu_ctx* c, float* t);
void bdpt_cpu_read_lightpaths(const bdpt_cpu_ctx* c, bdpt_lightpath* lp);
void bdpt_cpu_write_lightpaths(bdpt_cpu_ctx* c, const bdpt_lightpath* lp);
void bdpt_cpu_update_pixels(bdpt_cpu_ctx* c);
void bdpt_cpu_write_radiance(bdpt_cpu_ctx* c, const bdpt_vec* colors, const unsigned* counter);

#endif
