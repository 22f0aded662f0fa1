/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Nothing in the product (libsemtsdf.so, the
 * semtsdf Python host) links, imports or calls this file.  It is used only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
 *
 * Scalar C restatement of the reference fusion hot path of qq456cvb/SLAM-MaskRCNN, written
 * from the reference's text (not copied), with the f32 operation order the build defines
 * (DESIGN.md "floating-point contract"): compiled with -ffp-contract=off, fused
 * multiply-adds written out with fmaf(), IEEE division, so its f32 results are the bit
 * level reference for the HIP kernels.
 *
 * Followed reference locations:
 *   oracle_integrate         src/SfM_CUDA/tsdf.cu:18-70 (histogram, gate) and
 *                            src/TSDF_Python/tsdf.cu:10-58 (i32 colour ungated, label vote)
 *   oracle_project           the pixel choice of oracle_integrate (tsdf.cu:30-44)
 *   oracle_march_probs       src/SfM_CUDA/tsdf.cu:72-135, utils.cu:93-119,144-170
 *   oracle_filter_overlaps   src/SfM_CUDA/tsdf.cu:304-416 (+ configuration.h:8)
 *   oracle_render            src/SfM_CUDA/viewer.cu:17-86, palette viewer.cu:93-126
 *   oracle_place             src/SfM_CUDA/tsdf.cu:173-199 and src/TSDF_Python/tsdf.py:32-47
 *   oracle_orbit_camera      src/SfM_CUDA/viewer.cu:140-146
 *   oracle_shard_render_step the Z-sharded split of the march above (no reference counterpart)
 * Where the reference reads out of range (trilinear neighbours at the far faces,
 * utils.cu:103-113) the oracle clamps indices to the volume, which is the semantics the
 * build defines for that case.
 */
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OMAX 32

/* ---------------------------------------------------------------- helpers */
static int o_f2i_rd(float x) {
    float f = floorf(x);
    if (!(f == f)) return 0;
    if (f >= 2147483648.0f) return INT_MAX;
    if (f <= -2147483648.0f) return INT_MIN;
    return (int)f;
}

static float o_dot3(float a0, float a1, float a2, float b0, float b1, float b2) {
    float acc = a0 * b0;
    acc = fmaf(a1, b1, acc);
    return fmaf(a2, b2, acc);
}

static float o_mix(float a, float b, float t) { return fmaf(t, b, (1.0f - t) * a); }

/* geometry block shared by the entry points
 * geo[0..2] vol_start, geo[3..5] voxel, geo[6] mu, geo[7] depth_scale, geo[8] gate,
 * geo[9..11] vol_end */
typedef struct {
    int dx, dy, dz;
    float start[3], voxel[3], end[3];
    float mu, depth_scale, gate;
} ogeom;

static ogeom mk_geom(const int32_t* dims, const float* geo) {
    ogeom g;
    g.dx = dims[0]; g.dy = dims[1]; g.dz = dims[2];
    for (int i = 0; i < 3; ++i) { g.start[i] = geo[i]; g.voxel[i] = geo[3 + i]; g.end[i] = geo[9 + i]; }
    g.mu = geo[6]; g.depth_scale = geo[7]; g.gate = geo[8];
    return g;
}

/* ---------------------------------------------------------------- integrate
 * flags: 1 semantic histogram, 2 gate colour/hist on f < gate, 4 colour int32, 8 vote.
 * State arrays in reference layouts: sdf/wt/cls/cls_cnt [N], colour [N*3], hist
 * voxel-major [N*32].  Processes x in [x_begin, x_end).  counts[0] += touched,
 * counts[1] += gated, counts[2] += labels >= 32 seen (skipped). */
static void integrate_core(const int32_t* dims, const float* geo, const float* K9, const float* E16, int width,
                           int height, uint32_t flags, float* sdf, int32_t* wt, void* color, uint32_t* hist,
                           int32_t* cls, int32_t* cls_cnt, const uint16_t* depth, const uint8_t* rgb,
                           const uint8_t* mask, const int32_t* cls_in, int x_begin, int x_end, uint64_t* counts,
                           const int32_t* zmap, int lz, int x_state0);

void oracle_integrate(const int32_t* dims, const float* geo, const float* K9, const float* E16, int width,
                      int height, uint32_t flags, float* sdf, int32_t* wt, void* color, uint32_t* hist,
                      int32_t* cls, int32_t* cls_cnt, const uint16_t* depth, const uint8_t* rgb,
                      const uint8_t* mask, const int32_t* cls_in, int x_begin, int x_end, uint64_t* counts,
                      const int32_t* zmap, int lz) {
    integrate_core(dims, geo, K9, E16, width, height, flags, sdf, wt, color, hist, cls, cls_cnt, depth, rgb, mask,
                   cls_in, x_begin, x_end, counts, zmap, lz, 0);
}

/* The same over x-planes [x_begin, x_end) with state arrays that hold only those planes
 * ([x_end - x_begin][dims[1]][dims[2]]): slabs of volumes too large for a whole host copy
 * (1024^3), computed with the global voxel coordinates, so bit-identical to the full run. */
void oracle_integrate_slab(const int32_t* dims, const float* geo, const float* K9, const float* E16, int width,
                           int height, uint32_t flags, float* sdf, int32_t* wt, void* color, uint32_t* hist,
                           int32_t* cls, int32_t* cls_cnt, const uint16_t* depth, const uint8_t* rgb,
                           const uint8_t* mask, const int32_t* cls_in, int x_begin, int x_end, uint64_t* counts) {
    integrate_core(dims, geo, K9, E16, width, height, flags, sdf, wt, color, hist, cls, cls_cnt, depth, rgb, mask,
                   cls_in, x_begin, x_end, counts, NULL, 0, x_begin);
}

static void integrate_core(const int32_t* dims, const float* geo, const float* K9, const float* E16, int width,
                           int height, uint32_t flags, float* sdf, int32_t* wt, void* color, uint32_t* hist,
                           int32_t* cls, int32_t* cls_cnt, const uint16_t* depth, const uint8_t* rgb,
                           const uint8_t* mask, const int32_t* cls_in, int x_begin, int x_end, uint64_t* counts,
                           const int32_t* zmap, int lz, int x_state0) {
    /* zmap: global z of each of the lz local planes (a Z-slab shard); NULL =
       the whole volume.  State arrays are [dims[0]][dims[1]][lz], their plane 0 being
       x = x_state0. */
    const ogeom g = mk_geom(dims, geo);
    if (!zmap) lz = g.dz;
    const int sem = flags & 1, gate = flags & 2, ci32 = flags & 4, vote = flags & 8;
    uint64_t n_touch = 0, n_gate = 0, n_bad = 0;
    /* Screen map of the build's f32 contract: proj = E[0:3] . (p, 1) and
       screen = K . proj (tsdf.cu:31-39) are folded into s = M p + m, M = RN(K E3) and
       m = RN(K t), each entry a left-to-right sum of three double products rounded once;
       every affine row is evaluated as aff(r, c, p) = fma(r2, pz, fma(r1, py, fma(r0, px, c))). */
    float M[9], m[3];
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j)
            M[i * 3 + j] = (float)((double)K9[i * 3 + 0] * (double)E16[0 * 4 + j] +
                                   (double)K9[i * 3 + 1] * (double)E16[1 * 4 + j] +
                                   (double)K9[i * 3 + 2] * (double)E16[2 * 4 + j]);
        m[i] = (float)((double)K9[i * 3 + 0] * (double)E16[3] + (double)K9[i * 3 + 1] * (double)E16[7] +
                       (double)K9[i * 3 + 2] * (double)E16[11]);
    }
    for (int x = x_begin; x < x_end; ++x) {
        const float px = fmaf((float)x, g.voxel[0], g.start[0]);
        for (int y = 0; y < g.dy; ++y) {
            const float py = fmaf((float)y, g.voxel[1], g.start[1]);
            for (int z = 0; z < lz; ++z) {
                const int gz = zmap ? zmap[z] : z;
                if (gz >= g.dz) continue;
                const float pz = fmaf((float)gz, g.voxel[2], g.start[2]);
                /* camera depth proj.z (tsdf.cu:31-34) and screen position (tsdf.cu:35-39) */
                const float qz = fmaf(E16[10], pz, fmaf(E16[9], py, fmaf(E16[8], px, E16[11])));
                const float sx = fmaf(M[2], pz, fmaf(M[1], py, fmaf(M[0], px, m[0])));
                const float sy = fmaf(M[5], pz, fmaf(M[4], py, fmaf(M[3], px, m[1])));
                const float sz = fmaf(M[8], pz, fmaf(M[7], py, fmaf(M[6], px, m[2])));
                /* perspective divide and floor (tsdf.cu:40-44) */
                const int ix = o_f2i_rd(sx / sz);
                const int iy = o_f2i_rd(sy / sz);
                if (ix < 0 || ix >= width || iy < 0 || iy >= height) continue;
                const size_t img = (size_t)iy * width + ix;
                const uint16_t draw = depth[img];
                if (draw == 0) continue;
                float diff = (float)draw / g.depth_scale - qz; /* z difference (tsdf.cu:49) */
                if (diff <= -g.mu) continue;
                if (diff > g.mu) diff = g.mu;
                diff = diff / g.mu;
                const size_t v = ((size_t)(x - x_state0) * g.dy + y) * lz + z;
                const int w = wt[v];
                /* running mean with unit weight (tsdf.cu:56) */
                sdf[v] = fmaf(sdf[v], (float)w, diff) / (float)(w + 1);
                ++n_touch;
                if (!gate || diff < g.gate) {
                    ++n_gate;
                    for (int c = 0; c < 3; ++c) {
                        if (ci32) {
                            int32_t* col = (int32_t*)color;
                            col[v * 3 + c] = (col[v * 3 + c] * w + (int)rgb[img * 3 + c]) / (w + 1);
                        } else {
                            uint8_t* col = (uint8_t*)color;
                            /* int arithmetic of tsdf.cu:59; c * w wraps past 2^31 (w > 8.4 M)
                               as on the reference's hardware (explicitly, not as C UB) */
                            const int num = (int)((uint32_t)col[v * 3 + c] * (uint32_t)w + (uint32_t)rgb[img * 3 + c]);
                            col[v * 3 + c] = (uint8_t)(num / (w + 1));
                        }
                    }
                    if (sem) {
                        const unsigned lab = mask[img];
                        if (lab < OMAX) hist[v * OMAX + lab] += 1u;
                        else ++n_bad;
                    }
                }
                wt[v] = w + 1;
                if (vote) { /* TSDF_Python/tsdf.cu:48-57 */
                    const int lab = cls_in[img];
                    if (cls_cnt[v] == 0) {
                        cls[v] = lab;
                        cls_cnt[v] = 1;
                    } else if (cls[v] == lab) {
                        cls_cnt[v] += 1;
                    } else {
                        cls_cnt[v] -= 1;
                    }
                }
            }
        }
    }
    if (counts) { counts[0] += n_touch; counts[1] += n_gate; counts[2] += n_bad; }
}

/* Pixel each voxel of x-planes [x_begin, x_end) projects to under the same f32 contract as
 * oracle_integrate (y*width + x, or -1 off-image), flat x-major: tests use it to find the
 * voxels whose f32 pixel choice differs from the float64 reference block (tsdf.py:86-97). */
void oracle_project(const int32_t* dims, const float* geo, const float* K9, const float* E16, int width, int height,
                    int32_t* img_out, int x_begin, int x_end) {
    const ogeom g = mk_geom(dims, geo);
    float M[9], m[3];
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j)
            M[i * 3 + j] = (float)((double)K9[i * 3 + 0] * (double)E16[0 * 4 + j] +
                                   (double)K9[i * 3 + 1] * (double)E16[1 * 4 + j] +
                                   (double)K9[i * 3 + 2] * (double)E16[2 * 4 + j]);
        m[i] = (float)((double)K9[i * 3 + 0] * (double)E16[3] + (double)K9[i * 3 + 1] * (double)E16[7] +
                       (double)K9[i * 3 + 2] * (double)E16[11]);
    }
    for (int x = x_begin; x < x_end; ++x) {
        const float px = fmaf((float)x, g.voxel[0], g.start[0]);
        for (int y = 0; y < g.dy; ++y) {
            const float py = fmaf((float)y, g.voxel[1], g.start[1]);
            for (int z = 0; z < g.dz; ++z) {
                const float pz = fmaf((float)z, g.voxel[2], g.start[2]);
                const float sx = fmaf(M[2], pz, fmaf(M[1], py, fmaf(M[0], px, m[0])));
                const float sy = fmaf(M[5], pz, fmaf(M[4], py, fmaf(M[3], px, m[1])));
                const float sz = fmaf(M[8], pz, fmaf(M[7], py, fmaf(M[6], px, m[2])));
                const int ix = o_f2i_rd(sx / sz), iy = o_f2i_rd(sy / sz);
                const size_t v = ((size_t)x * g.dy + y) * g.dz + z;
                img_out[v] = (ix < 0 || ix >= width || iy < 0 || iy >= height) ? -1 : iy * width + ix;
            }
        }
    }
}

/* ---------------------------------------------------------------- trilinear samplers */
typedef struct {
    size_t idx[8]; /* d[i*4+j*2+k] -> flat voxel index */
    float fx, fy, fz;
} otri;

static int o_clamp(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

static otri o_tri(const ogeom* g, float px, float py, float pz) {
    otri t;
    const float ix = (px - g->start[0]) / g->voxel[0];
    const float iy = (py - g->start[1]) / g->voxel[1];
    const float iz = (pz - g->start[2]) / g->voxel[2];
    const int x = o_f2i_rd(ix), y = o_f2i_rd(iy), z = o_f2i_rd(iz);
    t.fx = ix - (float)x;
    t.fy = iy - (float)y;
    t.fz = iz - (float)z;
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int k = 0; k < 2; ++k) {
                const int xx = o_clamp(x + i, 0, g->dx - 1);
                const int yy = o_clamp(y + j, 0, g->dy - 1);
                const int zz = o_clamp(z + k, 0, g->dz - 1);
                t.idx[i * 4 + j * 2 + k] = ((size_t)xx * g->dy + yy) * g->dz + zz;
            }
    return t;
}

static float o_tri_eval(const float* d, const otri* t) {
    const float low = o_mix(o_mix(d[0], d[4], t->fx), o_mix(d[2], d[6], t->fx), t->fy);
    const float high = o_mix(o_mix(d[1], d[5], t->fx), o_mix(d[3], d[7], t->fx), t->fy);
    return o_mix(low, high, t->fz);
}

static float o_sample_sdf(const ogeom* g, const float* sdf, float px, float py, float pz) {
    const otri t = o_tri(g, px, py, pz);
    float d[8];
    for (int k = 0; k < 8; ++k) d[k] = sdf[t.idx[k]];
    return o_tri_eval(d, &t);
}

static void o_sample_hist(const ogeom* g, const uint32_t* hist, float px, float py, float pz, float* out) {
    const otri t = o_tri(g, px, py, pz);
    for (int b = 0; b < OMAX; ++b) {
        float d[8];
        for (int k = 0; k < 8; ++k) d[k] = (float)hist[t.idx[k] * OMAX + b];
        out[b] = o_tri_eval(d, &t);
    }
}

/* ray march shared by back_proj_kernel and show_tsdf_kernel */
static int o_march(const ogeom* g, const float* sdf, float ox, float oy, float oz, float dx, float dy, float dz,
                   float* t_hit) {
    const float ivx = 1.0f / dx, ivy = 1.0f / dy, ivz = 1.0f / dz;
    const float tbx = ivx * (g->start[0] - ox), tby = ivy * (g->start[1] - oy), tbz = ivz * (g->start[2] - oz);
    const float ttx = ivx * (g->end[0] - ox), tty = ivy * (g->end[1] - oy), ttz = ivz * (g->end[2] - oz);
    float tnear = fmaxf(fmaxf(fminf(ttx, tbx), fminf(tty, tby)), fminf(ttz, tbz));
    tnear = fmaxf(tnear, 0.01f);
    float tfar = fminf(fminf(fmaxf(ttx, tbx), fmaxf(tty, tby)), fmaxf(ttz, tbz));
    tfar = fminf(tfar, 100.0f);
    if (tnear > tfar) return 0;
    float t = tnear + 1e-6f;
    tfar -= 1e-6f;
    float f_tt = 0.0f, step = g->voxel[0];
    float f_t = o_sample_sdf(g, sdf, fmaf(t, dx, ox), fmaf(t, dy, oy), fmaf(t, dz, oz));
    if (!(f_t > 0.0f)) return 0;
    for (; t < tfar; t += step) {
        f_tt = o_sample_sdf(g, sdf, fmaf(t, dx, ox), fmaf(t, dy, oy), fmaf(t, dz, oz));
        if (f_tt < 0.0f) break;
        if (f_tt < g->voxel[0] / 2.0f) step = g->voxel[0] / 4.0f; /* sticky (tsdf.cu:116-119) */
        f_t = f_tt;
    }
    if (!(f_tt < 0.0f)) return 0;
    t += step * f_tt / (f_t - f_tt);
    *t_hit = t;
    return 1;
}

/* ---------------------------------------------------------------- association raycast
 * Kinv9: 3x3 of K^-1; E16: extrinsic2init.  Rt = E^T(3x3), o = -Rt t accumulated in
 * double (cv::gemm on CV_32F).  probs [H*W*32] and box [H*W*32] are fully written
 * (zeros where nothing is hit, like the memset of tsdf.cu:428-429). */
void oracle_march_probs(const int32_t* dims, const float* geo, const float* Kinv9, const float* E16, int width,
                        int height, const float* sdf, const uint32_t* hist, float box_thresh, float* probs,
                        uint8_t* box, int y_begin, int y_end) {
    const ogeom g = mk_geom(dims, geo);
    float Rt[9], o[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Rt[i * 3 + j] = E16[j * 4 + i];
    for (int i = 0; i < 3; ++i) {
        const double acc = (double)Rt[i * 3] * E16[3] + (double)Rt[i * 3 + 1] * E16[7] + (double)Rt[i * 3 + 2] * E16[11];
        o[i] = -(float)acc;
    }
    for (int y = y_begin; y < y_end; ++y)
        for (int x = 0; x < width; ++x) {
            const size_t px = (size_t)y * width + x;
            float* p = probs + px * OMAX;
            uint8_t* b = box + px * OMAX;
            memset(p, 0, sizeof(float) * OMAX);
            memset(b, 0, OMAX);
            const float fx = (float)x, fy = (float)y;
            const float tx = o_dot3(Kinv9[0], Kinv9[1], Kinv9[2], fx, fy, 1.0f);
            const float ty = o_dot3(Kinv9[3], Kinv9[4], Kinv9[5], fx, fy, 1.0f);
            const float tz = o_dot3(Kinv9[6], Kinv9[7], Kinv9[8], fx, fy, 1.0f);
            const float rx = o_dot3(Rt[0], Rt[1], Rt[2], tx, ty, tz);
            const float ry = o_dot3(Rt[3], Rt[4], Rt[5], tx, ty, tz);
            const float rz = o_dot3(Rt[6], Rt[7], Rt[8], tx, ty, tz);
            const float inv = 1.0f / sqrtf(o_dot3(rx, ry, rz, rx, ry, rz));
            const float dx = rx * inv, dy = ry * inv, dz = rz * inv;
            float t;
            if (!o_march(&g, sdf, o[0], o[1], o[2], dx, dy, dz, &t)) continue;
            o_sample_hist(&g, hist, fmaf(t, dx, o[0]), fmaf(t, dy, o[1]), fmaf(t, dz, o[2]), p);
            for (int k = 0; k < OMAX; ++k) b[k] = p[k] > box_thresh ? 1 : 0;
        }
}

/* ---------------------------------------------------------------- filter_overlaps
 * precision 0: the reference's float accumulation in pixel order (logf, expf) -- the rule the
 *   device reproduces;
 * precision 1: double accumulation of the same f32 terms, exp in double: a different rule,
 *   used by the tests to find the cases that f32 rounding decides.
 * mask is relabelled in place; *num_objs is updated.  assigned_prev[i] = previous id
 * matched by current label i (or -1), assigned_prob[i] its probability.
 * id_policy 0: new ids num_objs++ without a bound, stored in the u8 mask modulo 256 (tsdf.cu:379-383:
 *   mask_ptr[i] = num_objs, extra_assign is a uint8 map); 1: the engine's opt-in deviation
 *   SEMTSDF_F_ID_SATURATE -- a new id that would be >= 32 is 0 (background), num_objs stops at 32.
 * Returns max_obj_now. */
int oracle_filter_overlaps(const float* probs, const uint8_t* box, uint8_t* mask, int width, int height,
                           uint32_t n_obs, float eps, int precision, int* num_objs, int32_t* assigned_prev,
                           float* assigned_prob, double* prob_table, int id_policy) {
    const size_t n = (size_t)width * height;
    int maxv = 0;
    for (size_t i = 0; i < n; ++i)
        if (mask[i] > maxv) maxv = mask[i];
    const int max_obj_now = maxv + 1;
    static float af[OMAX][OMAX];
    static double ad[OMAX][OMAX];
    static uint32_t cnts[OMAX][OMAX];
    memset(af, 0, sizeof(af));
    memset(ad, 0, sizeof(ad));
    memset(cnts, 0, sizeof(cnts));
    const float nf = (float)n_obs;
    for (size_t i = 0; i < n; ++i) {
        const int m = mask[i];
        if (m > 0 && m < OMAX) {
            for (int j = 1; j < OMAX; ++j) {
                const float r = probs[i * OMAX + j] / nf;
                const float q = r > eps ? r : eps;
                if (precision == 0) af[m][j] += logf(q);
                else ad[m][j] += (double)logf(q);
                cnts[m][j]++;
            }
        }
        for (int nn = 1; nn < OMAX; ++nn) {
            if (!box[i * OMAX + nn]) continue;
            const float r = 1.0f - probs[i * OMAX + nn] / nf;
            const float q = r > eps ? r : eps;
            const float L = logf(q);
            for (int mm = 1; mm < max_obj_now && mm < OMAX; ++mm) {
                if (m == mm) continue;
                if (precision == 0) af[mm][nn] += L;
                else ad[mm][nn] += (double)L;
                cnts[mm][nn]++;
            }
        }
    }
    /* decisions: argmax_j exp(A/C), accept > 3 eps, keep the best current label per j */
    int map_i[OMAX];
    double map_p[OMAX];
    for (int j = 0; j < OMAX; ++j) { map_i[j] = -1; map_p[j] = 0.0; }
    for (int i = 0; i < OMAX; ++i) { assigned_prev[i] = -1; assigned_prob[i] = 0.0f; }
    const float thr = 3.0f * eps;
    for (int i = 1; i < max_obj_now && i < OMAX; ++i) {
        int max_j = -1;
        double max_p = 0.0;
        for (int j = 1; j < OMAX; ++j) {
            double prob;
            if (cnts[i][j] == 0) prob = 0.0;
            else if (precision == 0) prob = (double)expf(af[i][j] / (float)cnts[i][j]);
            else prob = exp(ad[i][j] / (double)cnts[i][j]);
            if (precision == 0) prob = (double)(float)prob;
            if (prob_table) prob_table[i * OMAX + j] = prob;  /* the candidates, for margins */
            if (prob > max_p) { max_j = j; max_p = prob; }
        }
        if (max_p > (double)thr) {
            if (map_i[max_j] < 0 || map_p[max_j] < max_p) { map_i[max_j] = i; map_p[max_j] = max_p; }
        }
    }
    int rev[256];
    for (int v = 0; v < 256; ++v) rev[v] = -1;
    for (int j = 0; j < OMAX; ++j)
        if (map_i[j] >= 0) {
            rev[map_i[j]] = j;
            assigned_prev[map_i[j]] = j;
            assigned_prob[map_i[j]] = (float)map_p[j];
        }
    int extra[256];
    for (int v = 0; v < 256; ++v) extra[v] = -1;
    int no = *num_objs;
    for (size_t i = 0; i < n; ++i) {
        const int m = mask[i];
        if (rev[m] >= 0) {
            mask[i] = (uint8_t)rev[m];
        } else if (m > 0) {
            if (extra[m] < 0) {
                if (id_policy == 1 && no >= OMAX) {
                    extra[m] = 0;  /* saturated: background */
                } else {
                    extra[m] = (uint8_t)no;
                    ++no;
                }
                mask[i] = (uint8_t)extra[m];
            } else {
                mask[i] = (uint8_t)extra[m];
            }
        }
    }
    *num_objs = no;
    return max_obj_now;
}

/* ---------------------------------------------------------------- render */
static const uint8_t o_palette[OMAX * 3] = {
    230, 25, 75, 60, 180, 75, 255, 225, 25, 0, 130, 200, 245, 130, 48, 145, 30, 180, 70, 240, 240, 240, 50, 230,
    210, 245, 60, 250, 190, 190, 0, 128, 128, 230, 190, 255, 170, 110, 40, 255, 250, 200, 128, 0, 0, 170, 255, 195,
    230, 25, 75, 60, 180, 75, 255, 225, 25, 0, 130, 200, 245, 130, 48, 145, 30, 180, 70, 240, 240, 240, 50, 230,
    210, 245, 60, 250, 190, 190, 0, 128, 128, 230, 190, 255, 170, 110, 40, 255, 250, 200, 128, 0, 0, 170, 255, 195};

/* mode 0 label (argmax histogram -> palette BGR), 1 colour at the hit.  s2w 4x4, c[3]. */
void oracle_render(const int32_t* dims, const float* geo, const float* s2w, const float* c, int width, int height,
                   int mode, int color_i32, const float* sdf, const uint32_t* hist, const void* color,
                   uint8_t* out_bgr, float* out_t, int y_begin, int y_end) {
    const ogeom g = mk_geom(dims, geo);
    for (int y = y_begin; y < y_end; ++y)
        for (int x = 0; x < width; ++x) {
            const size_t px = (size_t)y * width + x;
            uint8_t* o = out_bgr + px * 3;
            o[0] = o[1] = o[2] = 0;
            if (out_t) out_t[px] = -1.0f;
            const float fx = (float)x, fy = (float)y;
            const float tx = o_dot3(s2w[0], s2w[1], s2w[2], fx, fy, 1.0f) + s2w[3];
            const float ty = o_dot3(s2w[4], s2w[5], s2w[6], fx, fy, 1.0f) + s2w[7];
            const float tz = o_dot3(s2w[8], s2w[9], s2w[10], fx, fy, 1.0f) + s2w[11];
            const float rx = tx - c[0], ry = ty - c[1], rz = tz - c[2];
            const float inv = 1.0f / sqrtf(o_dot3(rx, ry, rz, rx, ry, rz));
            const float dx = rx * inv, dy = ry * inv, dz = rz * inv;
            float t;
            if (!o_march(&g, sdf, c[0], c[1], c[2], dx, dy, dz, &t)) continue;
            if (out_t) out_t[px] = t;
            const float hx = fmaf(t, dx, c[0]), hy = fmaf(t, dy, c[1]), hz = fmaf(t, dz, c[2]);
            if (mode == 0) {
                float cnt[OMAX];
                o_sample_hist(&g, hist, hx, hy, hz, cnt);
                float best = 0.0f;
                int obj = 0;
                for (int k = 0; k < OMAX; ++k)
                    if (cnt[k] > best) { best = cnt[k]; obj = k; }
                if (obj > 0) {
                    o[0] = o_palette[obj * 3 + 2];
                    o[1] = o_palette[obj * 3 + 1];
                    o[2] = o_palette[obj * 3 + 0];
                }
            } else {
                const otri tr = o_tri(&g, hx, hy, hz);
                for (int ch = 0; ch < 3; ++ch) {
                    float d[8];
                    for (int k = 0; k < 8; ++k)
                        d[k] = color_i32 ? (float)((const int32_t*)color)[tr.idx[k] * 3 + ch]
                                         : (float)((const uint8_t*)color)[tr.idx[k] * 3 + ch];
                    o[ch] = (uint8_t)(int)o_tri_eval(d, &tr);
                }
            }
        }
}

/* ---------------------------------------------------------------- Z-sharded render
 * Restatement of the sharded raycast protocol (k_shard_ray_step / k_shard_render_final /
 * k_shard_render_finish in semtsdf_kernels.hip) for the tests: virtual shard `shard` of
 * `nshards` (chunks of `chunk` planes dealt round by round in boustrophedon order: shard s
 * owns position s of even rounds, n - 1 - s of odd ones) evaluates only the samples whose
 * base plane it owns; sampling reads the full volume, which equals the shard's local copy
 * (halo planes are integrated identically).  Records are int32 pairs {key, value bits};
 * the combine is the minimum key over shards.  state: 6 x npx words (k, fk, j, fj, fp, t).
 * step 0..3 as in the kernels; step 4 = composite (gathered of step 3 -> out_bgr/out_t). */
static int o_owner(const ogeom* g, float pz, int chunk, int nshards) {
    const float iz = (pz - g->start[2]) / g->voxel[2];
    const int zc = o_clamp(o_f2i_rd(iz), 0, g->dz - 1);
    const int c = zc / chunk, r = c / nshards, k = c - r * nshards;
    return (r & 1) ? nshards - 1 - k : k;
}

static void o_gmin(const int32_t* gth, int n, size_t npx, size_t px, int32_t* key, int32_t* val) {
    int32_t bk = INT_MAX, bv = 0;
    for (int r = 0; r < n; ++r) {
        const int32_t k = gth[((size_t)r * npx + px) * 2], v = gth[((size_t)r * npx + px) * 2 + 1];
        if (k < bk) { bk = k; bv = v; }
    }
    *key = bk;
    *val = bv;
}

static float o_bits_f(int32_t v) { float f; memcpy(&f, &v, 4); return f; }
static int32_t o_f_bits(float f) { int32_t v; memcpy(&v, &f, 4); return v; }

static float o_replay(float t, int ncoarse, int nfine, float vx) {
    for (int i = 0; i < ncoarse; ++i) t += vx;
    const float q = vx / 4.0f;
    for (int i = 0; i < nfine; ++i) t += q;
    return t;
}

void oracle_shard_render_step(const int32_t* dims, const float* geo, const float* s2w, const float* c, int width,
                              int height, int mode, int color_i32, const float* sdf, const uint32_t* hist,
                              const void* color, int step, int shard, int nshards, int chunk,
                              const int32_t* gathered, int32_t* send, int32_t* state, uint8_t* out_bgr,
                              float* out_t) {
    const ogeom g = mk_geom(dims, geo);
    const size_t npx = (size_t)width * height;
    int32_t* sk = state;
    float* sfk = (float*)(state + npx);
    int32_t* sj = state + 2 * npx;
    float* sfj = (float*)(state + 3 * npx);
    float* sfp = (float*)(state + 4 * npx);
    float* st = (float*)(state + 5 * npx);
    const float vx = g.voxel[0];
    for (int y = 0; y < height; ++y)
        for (int x = 0; x < width; ++x) {
            const size_t px = (size_t)y * width + x;
            if (step == 4) {
                int32_t k, v;
                o_gmin(gathered, nshards, npx, px, &k, &v);
                out_bgr[px * 3 + 0] = (uint8_t)(v & 0xFF);
                out_bgr[px * 3 + 1] = (uint8_t)((v >> 8) & 0xFF);
                out_bgr[px * 3 + 2] = (uint8_t)((v >> 16) & 0xFF);
                if (out_t) out_t[px] = st[px];
                continue;
            }
            const float fx = (float)x, fy = (float)y;
            const float tx = o_dot3(s2w[0], s2w[1], s2w[2], fx, fy, 1.0f) + s2w[3];
            const float ty = o_dot3(s2w[4], s2w[5], s2w[6], fx, fy, 1.0f) + s2w[7];
            const float tz = o_dot3(s2w[8], s2w[9], s2w[10], fx, fy, 1.0f) + s2w[11];
            const float rx = tx - c[0], ry = ty - c[1], rz = tz - c[2];
            const float inv = 1.0f / sqrtf(o_dot3(rx, ry, rz, rx, ry, rz));
            const float dx = rx * inv, dy = ry * inv, dz = rz * inv;
            const float ox = c[0], oy = c[1], oz = c[2];
            /* slab test of o_march */
            const float ivx = 1.0f / dx, ivy = 1.0f / dy, ivz = 1.0f / dz;
            const float tbx = ivx * (g.start[0] - ox), tby = ivy * (g.start[1] - oy), tbz = ivz * (g.start[2] - oz);
            const float ttx = ivx * (g.end[0] - ox), tty = ivy * (g.end[1] - oy), ttz = ivz * (g.end[2] - oz);
            float tnear = fmaxf(fmaxf(fminf(ttx, tbx), fminf(tty, tby)), fminf(ttz, tbz));
            tnear = fmaxf(tnear, 0.01f);
            float tfar = fminf(fminf(fmaxf(ttx, tbx), fmaxf(tty, tby)), fmaxf(ttz, tbz));
            tfar = fminf(tfar, 100.0f);
            const int in = !(tnear > tfar);
            const float t0 = tnear + 1e-6f, t1 = tfar - 1e-6f;
#define OWNS(t) (o_owner(&g, fmaf((t), dz, oz), chunk, nshards) == shard)
#define SAMPLE(t) o_sample_sdf(&g, sdf, fmaf((t), dx, ox), fmaf((t), dy, oy), fmaf((t), dz, oz))
            int32_t rk = INT_MAX, rv = 0;
            if (step == 0) {
                if (!in) {
                    rk = -1;
                } else {
                    float t = t0;
                    int dead = 0;
                    if (OWNS(t) && !(SAMPLE(t) > 0.0f)) { rk = -1; dead = 1; }
                    if (!dead) {
                        if (!(t < t1)) rk = -1;
                        else
                            for (int k = 0; t < t1; ++k, t += vx) {
                                if (!OWNS(t)) continue;
                                const float f = SAMPLE(t);
                                if (f < vx / 2.0f) { rk = k; rv = o_f_bits(f); break; }
                            }
                    }
                }
            } else if (step == 1) {
                int32_t k, v;
                o_gmin(gathered, nshards, npx, px, &k, &v);
                if (k < 0 || k == INT_MAX) {
                    sk[px] = -1;
                } else {
                    const float fk = o_bits_f(v);
                    sk[px] = k;
                    sfk[px] = fk;
                    if (fk < 0.0f) {
                        sj[px] = 0;
                        const float t = o_replay(t0, k - 1, 0, vx);
                        if (OWNS(t)) { rk = 0; rv = o_f_bits(SAMPLE(t)); }
                    } else {
                        float t = o_replay(t0, k, 0, vx);
                        const float q = vx / 4.0f;
                        for (int j = 1;; ++j) {
                            t += q;
                            if (!(t < t1)) break;
                            if (!OWNS(t)) continue;
                            const float f = SAMPLE(t);
                            if (f < 0.0f) { rk = j; rv = o_f_bits(f); break; }
                        }
                    }
                }
            } else if (step == 2) {
                const int k = sk[px];
                if (k >= 0) {
                    int32_t ck, cv;
                    o_gmin(gathered, nshards, npx, px, &ck, &cv);
                    if (sfk[px] < 0.0f) {
                        sfp[px] = o_bits_f(cv);
                    } else if (ck == INT_MAX) {
                        sk[px] = -1;
                    } else {
                        sj[px] = ck;
                        sfj[px] = o_bits_f(cv);
                        if (ck == 1) {
                            sfp[px] = sfk[px];
                        } else {
                            const float t = o_replay(t0, k, ck - 1, vx);
                            if (OWNS(t)) { rk = 0; rv = o_f_bits(SAMPLE(t)); }
                        }
                    }
                }
            } else { /* step 3: resolve the hit, shade by the owner of the hit point */
                const int k = sk[px];
                if (k < 0) {
                    st[px] = -1.0f;
                    if (shard == 0) { rk = 0; rv = 0; }
                } else {
                    float ts, stp, f, fp;
                    if (sfk[px] < 0.0f) {
                        ts = o_replay(t0, k, 0, vx);
                        stp = vx;
                        f = sfk[px];
                        fp = sfp[px];
                    } else {
                        const int j = sj[px];
                        if (j >= 2) {
                            int32_t ck, cv;
                            o_gmin(gathered, nshards, npx, px, &ck, &cv);
                            sfp[px] = o_bits_f(cv);
                        }
                        ts = o_replay(t0, k, j, vx);
                        stp = vx / 4.0f;
                        f = sfj[px];
                        fp = sfp[px];
                    }
                    const float t = ts + stp * f / (fp - f);
                    st[px] = t;
                    const float hx = fmaf(t, dx, ox), hy = fmaf(t, dy, oy), hz = fmaf(t, dz, oz);
                    if (o_owner(&g, hz, chunk, nshards) == shard) {
                        uint8_t o[3] = {0, 0, 0};
                        if (mode == 0) {
                            float cnt[OMAX];
                            o_sample_hist(&g, hist, hx, hy, hz, cnt);
                            float best = 0.0f;
                            int obj = 0;
                            for (int b = 0; b < OMAX; ++b)
                                if (cnt[b] > best) { best = cnt[b]; obj = b; }
                            if (obj > 0) {
                                o[0] = o_palette[obj * 3 + 2];
                                o[1] = o_palette[obj * 3 + 1];
                                o[2] = o_palette[obj * 3 + 0];
                            }
                        } else {
                            const otri tr = o_tri(&g, hx, hy, hz);
                            for (int ch = 0; ch < 3; ++ch) {
                                float d[8];
                                for (int kk = 0; kk < 8; ++kk)
                                    d[kk] = color_i32 ? (float)((const int32_t*)color)[tr.idx[kk] * 3 + ch]
                                                      : (float)((const uint8_t*)color)[tr.idx[kk] * 3 + ch];
                                o[ch] = (uint8_t)(int)o_tri_eval(d, &tr);
                            }
                        }
                        rk = 0;
                        rv = (int32_t)((uint32_t)o[0] | ((uint32_t)o[1] << 8) | ((uint32_t)o[2] << 16));
                    }
                }
            }
#undef OWNS
#undef SAMPLE
            send[px * 2] = rk;
            send[px * 2 + 1] = rv;
        }
}

/* ---------------------------------------------------------------- placement
 * mode 0 SfM (f32, saturating u8 mask, mean in metres), 1 TSDF_Python (f64, wrapping u8
 * mask, mean in raw units).  Kinv16 row-major.  out: start[3], end[3], voxel[3], mu. */
int oracle_place(const uint16_t* depth, int width, int height, const float* Kinv16, const int32_t* dims,
                 double mean_depth, int mode, float* out10) {
    int x0 = width, y0 = height, x1 = -1, y1 = -1;
    for (int y = 0; y < height; ++y)
        for (int x = 0; x < width; ++x) {
            const uint16_t d = depth[(size_t)y * width + x];
            const int nz = mode == 1 ? ((uint8_t)d != 0) : (d != 0);
            if (!nz) continue;
            if (x < x0) x0 = x;
            if (x > x1) x1 = x;
            if (y < y0) y0 = y;
            if (y > y1) y1 = y;
        }
    if (x1 < 0) return -1;
    const double tlp[3] = {x0, y0, 1.0}, brp[3] = {x1 + 1, y1 + 1, 1.0};
    if (mode == 1) {
        const double md = mean_depth / 5000.0;
        double tl[3], br[3], vox0 = 0;
        for (int i = 0; i < 3; ++i) {
            tl[i] = ((double)Kinv16[i * 4] * tlp[0] + (double)Kinv16[i * 4 + 1] * tlp[1]) + (double)Kinv16[i * 4 + 2];
            br[i] = ((double)Kinv16[i * 4] * brp[0] + (double)Kinv16[i * 4 + 1] * brp[1]) + (double)Kinv16[i * 4 + 2];
            tl[i] *= md;
            br[i] *= md;
        }
        const double ddx = tl[0] - br[0], ddy = tl[1] - br[1];
        const double half = sqrt(ddx * ddx + ddy * ddy) / 2.0;
        for (int i = 0; i < 3; ++i) {
            const double cc = (tl[i] + br[i]) / 2.0;
            const double s = cc - half, e = cc + half;
            const double vx = (e - s) / (double)(dims[i] - 1);
            out10[i] = (float)s;
            out10[3 + i] = (float)e;
            out10[6 + i] = (float)vx;
            if (i == 0) vox0 = vx;
        }
        out10[9] = (float)(5.0 * vox0);
    } else {
        const float md = (float)mean_depth;
        float tl[3], br[3];
        for (int i = 0; i < 3; ++i) {
            double at = 0, ab = 0;
            for (int k = 0; k < 4; ++k) {
                const double tv = k < 2 ? tlp[k] : 1.0, bv = k < 2 ? brp[k] : 1.0;
                at += (double)Kinv16[i * 4 + k] * tv;
                ab += (double)Kinv16[i * 4 + k] * bv;
            }
            tl[i] = (float)((double)(float)at * (double)md);
            br[i] = (float)((double)(float)ab * (double)md);
        }
        const float ddx = tl[0] - br[0], ddy = tl[1] - br[1];
        const float half = (float)(sqrt((double)ddx * (double)ddx + (double)ddy * (double)ddy) / 2.0);
        for (int i = 0; i < 3; ++i) {
            const float cc = (tl[i] + br[i]) * 0.5f;
            out10[i] = cc - half;
            out10[3 + i] = cc + half;
            out10[6 + i] = (out10[3 + i] - out10[i]) / (float)(dims[i] - 1);
        }
        out10[9] = 5.0f * out10[6];
    }
    return 0;
}

void oracle_orbit_camera(const float* Kinv16, float angle, float dist, float* s2w, float* c) {
    const float ca = cosf(angle), sa = sinf(angle);
    const float rot[16] = {ca, 0, -sa, dist * sa, 0, 1, 0, 0, sa, 0, ca, dist - dist * ca, 0, 0, 0, 1};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double acc = 0;
            for (int k = 0; k < 4; ++k) acc += (double)rot[i * 4 + k] * (double)Kinv16[k * 4 + j];
            s2w[i * 4 + j] = (float)acc;
        }
    const float r = dist + 0.5f;
    c[0] = r * sa;
    c[1] = 0.0f;
    c[2] = r - r * ca;
}

/* ---------------------------------------------------------------- division check
 * Test support for k_integrate's div_by_rcp: number of a[i] (|a| >= 2^-60) for which
 * RN(q0 + r y), q0 = RN(a y), r = fma(-q0, b, a), y = RN(1/b), differs from RN(a/b). */
int oracle_div_rcp_mismatches(const float* a, int n, float b) {
    const float y = 1.0f / b;
    int bad = 0;
    for (int i = 0; i < n; ++i) {
        const float x = a[i];
        if (!(fabsf(x) >= 0x1p-60f)) continue;
        const float q0 = x * y;
        const float r = fmaf(-q0, b, x);
        const float q1 = fmaf(r, y, q0);
        const float ref = x / b;
        if (memcmp(&q1, &ref, 4) != 0) ++bad;
    }
    return bad;
}

/* ---------------------------------------------------------------- libm check
 * Test support for the device's association log/exp (semtsdf_libm.h): number of i for which
 * y[i] differs in bits from this C library's logf(x[i]) (fn 0) or expf(x[i]) (fn 1) -- the
 * functions the reference's host filter_overlaps calls (tsdf.cu:318,329,343).  x[i] may be
 * NULL-generated: when x == NULL the inputs are the consecutive float bit patterns u0 + i. */
long oracle_libm_mismatches(int fn, const float* x, const float* y, long n, uint32_t u0) {
    long bad = 0;
    for (long i = 0; i < n; ++i) {
        float xi;
        if (x) {
            xi = x[i];
        } else {
            const uint32_t u = u0 + (uint32_t)i;
            memcpy(&xi, &u, 4);
        }
        const float r = fn == 0 ? logf(xi) : expf(xi);
        if (memcmp(&r, &y[i], 4) != 0) ++bad;
    }
    return bad;
}

/* Largest distance in ulps (of the library result) between y[i] and this C library's logf of
 * the consecutive float bit patterns u0 + i: bounds the device logf the association march's
 * fixed-point sums use (the certificate's term slack). */
double oracle_logf_ulp_max(const float* y, long n, uint32_t u0) {
    double worst = 0.0;
    for (long i = 0; i < n; ++i) {
        const uint32_t u = u0 + (uint32_t)i;
        float xi;
        memcpy(&xi, &u, 4);
        const float r = logf(xi);
        if (r == 0.0f) {
            if (y[i] != 0.0f) worst = INFINITY;
            continue;
        }
        const double d = fabs((double)y[i] - (double)r) / (double)(nextafterf(fabsf(r), INFINITY) - fabsf(r));
        if (d > worst) worst = d;
    }
    return worst;
}
