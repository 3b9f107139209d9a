/*
 * gs_oracle.h -- CPU ORACLE for the project -> bin -> sort -> blend frame path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (gaussian_splat_ipu_amd/,
 * include/) links, loads or calls this code.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may use it, and only as the checker / the
 * reported CPU baseline.
 *
 * It is an independent plain-C++ restatement of the reference rasteriser
 * (Nmjfry/gaussian_splat_ipu):
 *   - per-Gaussian math   include/splat/ipu_geometry.hpp:232-384
 *   - tile geometry       include/tileMapping/tile_config.hpp:19-71
 *   - viewport            include/splat/viewport.hpp:21-35
 *   - codelet             codelets/splat/codelets.cpp:358-421 (renderTile),
 *                         :437-505 (renderInternal), :605-639 (compute)
 *   - binning             the *converged* state of the tile lattice
 *                         (codelets.cpp:194-293,507-602)
 *   - readback            src/splat/ipu_rasteriser.cpp:115-144
 *   - CPU point path      src/splat/cpu_rasteriser.cpp:9-92
 * glm (absent from the reference snapshot, version unpinned) is restated with
 * glm 0.9.9 conventions: column-major m[c][r]; mat4*vec4 =
 * (m0*x + m1*y) + (m2*z + m3*w); mat*mat summed left to right.
 *
 * Pinning: the reference's own known-answer tests (tests/test.cpp:21-34,
 * codelets/tests/codelets.cpp:34-97) pin the matrix/tile arithmetic; the
 * covariance / binning / per-pixel results are NOT pinned by any reference
 * test or fixture (the reference has none and cannot be built here: Poplar,
 * glm, OpenCV absent).  Status: "parity partially pinned" -- see DESIGN.md.
 */
#ifndef GS_ORACLE_H
#define GS_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One frame's parameters.  Matrices are row-major on the wire, exactly as
 * IpuSplatter::updateModelView/updateProjection store them
 * (ipu_rasteriser.cpp:86-102). */
typedef struct or_frame {
  float view_rm[16];
  float proj_rm[16];
  float fov;            /* fxy[0] (radians, full angle)           */
  float scale_div;      /* fxy[1] (= lambda1/10 in splat.cpp:262)  */
  int32_t width, height;        /* IMWIDTH, IMHEIGHT              */
  int32_t tile_w, tile_h;       /* IPU_TILEWIDTH, IPU_TILEHEIGHT  */
  int32_t guard_tile_w, guard_tile_h; /* tile used by the guard band */
  float guard_band;             /* clipSize = 15 (codelets.cpp:622) */
  int32_t band_ty0, band_ty1;   /* tile-row band [ty0, ty1); 0,0 = all */
} or_frame;

/* Per-Gaussian result of the projection stage (rows a1-a8, a11). */
typedef struct or_proj {
  float mean2d[2];    /* Viewport::clipSpaceToViewport            */
  float cov2d[3];     /* Gaussian3D::ComputeCov2D                 */
  float conic[4];     /* Gaussian2D::ComputeConicOpacity          */
  float clip_z;       /* Gaussian2D::z (sort key)                 */
  float radius;       /* GetBoundingBox my_radius                 */
  int32_t rendered;   /* withinGuardBand && z < 0                 */
  int32_t rect[4];    /* tx0, ty0, tx1, ty1 inclusive, band-relative rows; empty if tx0>tx1 */
} or_proj;

typedef struct or_stats {
  int64_t n_rendered;   /* V */
  int64_t n_pairs;      /* P */
  int64_t max_list;     /* max_t L_t */
  int32_t n_tiles;      /* T */
  int32_t tiles_x, tiles_y;
} or_stats;

/* glm restatement entry points, column-major (for the reference KATs) */
void or_mat4_mul(const float* a, const float* b, float* out);
void or_mat4_mul_vec4(const float* m, const float* v, float* out);

/* portable expf shared (as an algorithm) with the HIP kernels */
float or_expf(float x);

/* per-frame scalars exactly as the codelet derives them (codelets.cpp:444-448) */
void or_frame_scalars(const or_frame* f, float* tanfov, float* focal_x, float* focal_y,
                      float* guard_thr);

int or_project(const float* g64, int64_t n, const or_frame* f, or_proj* out, int nthreads);

/* Converged binning: per band tile, the list of Gaussian indices sorted by
 * (clip z ascending, index ascending).  tile_start has T+1 entries.  Returns
 * P, or -1 if cap is too small (lists untouched beyond cap). */
int64_t or_bin(const or_proj* p, int64_t n, const or_frame* f, int64_t* tile_start,
               uint32_t* list, int64_t cap, int nthreads);

/* Blend every band tile into a row-major RGBA f32 image of the band rows
 * (width x band_pixel_rows x 4). */
int or_blend(const float* g64, const or_proj* p, const or_frame* f, const int64_t* tile_start,
             const uint32_t* list, float* rgba, int nthreads);

/* a14: min(v*255,255) -> round-half-even saturate -> RGBA2BGR, row-major */
void or_pack_bgr8(const float* rgba, int64_t n_pixels, uint8_t* bgr);

/* Whole frame.  rgba may be NULL.  hist (T entries) may be NULL. */
int or_render(const float* g64, int64_t n, const or_frame* f, float* rgba, uint8_t* bgr,
              uint32_t* hist, or_stats* st, int nthreads);

/* Restated CPU point-splat path (cpu_rasteriser.cpp:9-92): image is H x W x 3
 * u8 (zeroed by caller); returns splatted count.  hist may be NULL. */
/* Opt-in view-dependent colour (the product's gs_set_sh; the reference
 * itself reads f_dc only, file_io.cpp:66-68): out_g64 = g64 with every
 * Gaussian's colour.rgb replaced by the 3DGS spherical-harmonic colour of
 * degree 0..3 for the direction from campos to its mean (scene frame, z
 * negated back to the PLY frame), max(.., 0).  f_dc: n x 3, f_rest: n x 45
 * (channel-major), both in input order.  Not parity-pinned by the reference. */
void or_sh_colours(const float* g64, int64_t n, const float* f_dc, const float* f_rest, int degree,
                   const float campos[3], float* out_g64);
/* The camera position (scene frame) of a row-major view matrix [A t; 0 1]:
 * -A^-1 t in double, rounded once. */
void or_camera_position(const float* view_rm, float* campos);

/* The CPU the OpenMP team's threads run on: a parallel region of nthreads
 * threads (0 = the runtime's default), each spinning ~spin_ms so the team is
 * live at once, records sched_getcpu() into cpus[thread] (cap entries).
 * Returns the team size.  bench.py's CPU baseline reports the distinct CPUs
 * (and physical cores) of the team that actually ran. */
int or_omp_team_cpus(int nthreads, int* cpus, int cap, double spin_ms);
uint32_t or_point_splat(const float* xyz, int64_t n, const float* view_rm, const float* proj_rm,
                        int32_t width, int32_t height, int32_t tile_w, int32_t tile_h,
                        uint8_t* image, uint32_t* hist, int nthreads);


/* the lattice-migration emulator -- the reference's per-tile
 * codelet and channel exchange, one call per frame (codelets.cpp:143-641,
 * ipu_rasteriser.cpp:164-420, edge_builder.cpp:15-84).  Requires
 * width % tile_w == 0 and height % tile_h == 0 (the reference's macros).
 * Choices where the reference is undefined (unpinned): never-written memory
 * (padding slots, extra storage, in-channels before the first exchange, the
 * z-buffer) reads as zeros; `directions` outside the guard band are all false;
 * float -> unsigned of negative / NaN tile indices saturates to 0; z-buffer
 * reads past a tile's capacity (the last tile's is 600 entries shorter) are
 * empty records; the six workers of a tile do not race.  NULL on bad input. */
typedef struct or_lattice or_lattice;
or_lattice* or_lattice_create(const float* g64, int64_t n, const or_frame* f);
int or_lattice_step(or_lattice* L, const or_frame* f, int nthreads);
int64_t or_lattice_total_slots(const or_lattice* L);
/* rgba: width x height x 4 row-major; hist: the splatted counter per tile;
 * slot_gids: gid of every vertsIn slot (tile t's slots from t * (gpt + 600));
 * counters[6]: frames, dropped, send_failed, overrun (last frame), gpt, rem.
 * Any pointer may be NULL. */
void or_lattice_read(const or_lattice* L, float* rgba, uint32_t* hist, float* slot_gids, uint64_t* counters);
void or_lattice_destroy(or_lattice* L);

#ifdef __cplusplus
}
#endif
#endif
