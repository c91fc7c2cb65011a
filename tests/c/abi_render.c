/*
 * abi_render.c -- TEST: a plain-C host of the renderer's C ABI, calling
 * rt_render (include/rt_abi.h) the way INTEGRATION.md's cgo shim does: the
 * GML scene already flattened in BFS order (raytracer.go:776-828) with each
 * object's raw TransformMat (as the GML evaluator composes it,
 * existing.MulMat(new), evaluator.go:176-184), materials from
 * gml.Material, point lights, and -- for closure surfaces -- a surface
 * program hand-assembled from the bytecode contract in rt_abi.h.
 *
 *   abi_render canned  out.rgba   internal/gml/testdata/canned.gml (golden example_canned.png)
 *   abi_render sphere  out.rgba   internal/gml/testdata/sphere.gml (golden example_sphere.png)
 *   abi_render file scene.bin out.rgba host|peer [device ...]
 *       any flattened scene, read from the file go_raytracer_amd.scene.write_scene_file
 *       wrote (the rt_scene scalars and arrays as raw rt_abi.h structs), rendered by
 *       rt_render_ex (ABI 6) on the listed devices (repeats allowed; none = the
 *       current device) with the given gather
 *
 * Writes the width*height*4 image.RGBA.Pix bytes and prints the work counters
 * as one JSON line. Build: tests/hip/Makefile (links go-raytracer_amd/csrc/librtamd.so).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_abi.h"

static void translate_uscale(double *m, double tx, double ty, double tz, double s) {
    /* Translate(t) then Uscale(s) in GML order: TransformMat = T . S */
    memset(m, 0, 16 * sizeof(double));
    m[0] = m[5] = m[10] = s;
    m[3] = tx;
    m[7] = ty;
    m[11] = tz;
    m[15] = 1.0;
}

static rt_material mat(double r, double g, double b, double refl, double fuzz, double tr, double ior, double kd,
                       double ks, double n) {
    rt_material m;
    m.color[0] = r;
    m.color[1] = g;
    m.color[2] = b;
    m.reflectivity = refl;
    m.fuzziness = fuzz;
    m.transparency = tr;
    m.refractive_index = ior;
    m.kd = kd;
    m.ks = ks;
    m.specular_exponent = n;
    return m;
}

static int emit(const rt_scene *sc, const char *path) {
    size_t bytes = (size_t)sc->width * sc->height * 4;
    uint8_t *pix = (uint8_t *)malloc(bytes);
    rt_stats st;
    if (!pix) return 2;
    int rc = rt_render(sc, pix, &st);
    if (rc != RT_OK) {
        fprintf(stderr, "rt_render failed (%d): %s\n", rc, rt_last_error());
        free(pix);
        return 1;
    }
    FILE *f = fopen(path, "wb");
    if (!f || fwrite(pix, 1, bytes, f) != bytes) {
        fprintf(stderr, "cannot write %s\n", path);
        free(pix);
        return 2;
    }
    fclose(f);
    free(pix);
    printf("{\"width\": %d, \"height\": %d, \"primary_rays\": %llu, \"secondary_rays\": %llu, \"shadow_rays\": %llu, "
           "\"shaded_hits\": %llu, \"surface_errors\": %llu, \"sphere_tests\": %llu}\n",
           sc->width, sc->height, (unsigned long long)st.primary_rays, (unsigned long long)st.secondary_rays,
           (unsigned long long)st.shadow_rays, (unsigned long long)st.shaded_hits,
           (unsigned long long)st.surface_errors, (unsigned long long)st.tests[RT_SPHERE]);
    return 0;
}

/* canned.gml: green mirror, dull fuzzy, glass, ground sphere; BFS order of
 * union(union(union(ground, glass), dull), green). */
static int canned(const char *out) {
    rt_material mats[4] = {
        mat(0.2, 0.8, 0.2, 0.8, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0),  /* green: refl 0.8 */
        mat(0.2, 0.2, 0.8, 0.2, 0.5, 0.0, 0.0, 1.0, 0.0, 0.0),  /* dull: refl 0.2 fuzz 0.5 */
        mat(0.8, 0.2, 0.2, 0.0, 0.0, 0.9, 1.5, 1.0, 0.8, 50.0), /* glass */
        mat(0.8, 0.8, 0.8, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0),  /* ground: `color 1.0 0.0 0.0` surface, Reflectivity = ks */
    };
    rt_object objs[4];
    memset(objs, 0, sizeof objs);
    const double pos[4][4] = {{-2.0, 0.0, 6.0, 1.0}, {2.0, 0.0, 8.0, 1.0}, {0.0, 0.0, 5.0, 1.0}, {0.0, -1001.0, 5.0, 1000.0}};
    for (int i = 0; i < 4; i++) {
        objs[i].kind = RT_SPHERE;
        objs[i].has_transform = 1;
        translate_uscale(objs[i].transform, pos[i][0], pos[i][1], pos[i][2], pos[i][3]);
        for (int f = 0; f < RT_MAX_FACES; f++) objs[i].material[f] = i;
    }
    rt_point_light light = {{5.0, 5.0, 0.0}, {1.0, 1.0, 1.0}};
    rt_scene sc;
    memset(&sc, 0, sizeof sc);
    sc.width = 1900;
    sc.height = 1200;
    sc.depth = 7;
    sc.fov = 120.0;
    sc.ambient[0] = sc.ambient[1] = sc.ambient[2] = 0.1;
    sc.bg_end[0] = 0.5;
    sc.bg_end[1] = 0.7;
    sc.bg_end[2] = 1.0;
    sc.num_lights = 1;
    sc.lights = &light;
    sc.objects = objs;
    sc.num_objects = 4;
    sc.materials = mats;
    sc.num_materials = 4;
    return emit(&sc, out);
}

/* sphere.gml: one closure `{ /v /u /face 0.8 0.2 v point 1.0 0.2 1.0 }`
 * used by two spheres, hand-compiled to the rt_abi.h bytecode. */
static int sphere(const char *out) {
    union {
        double d;
        uint64_t u;
    } k[4];
    k[0].d = 0.8;
    k[1].d = 0.2;
    k[2].d = 0.0;
    k[3].d = 1.0;
    const uint64_t consts[4] = {k[0].u, k[1].u, k[2].u, k[3].u};
    const uint32_t code[] = {
        RT_VM_INSN(RT_VM_CONST, 0, 0, 0), 0,  /* colour r = 0.8 */
        RT_VM_INSN(RT_VM_CONST, 1, 0, 0), 1,  /* colour g = 0.2 */
        RT_VM_INSN(RT_VM_MOV, 2, 12, 0), 0,   /* colour b = v */
        RT_VM_INSN(RT_VM_CONST, 3, 0, 0), 1,  /* reflectivity = ks (EvalSurfaceFn) */
        RT_VM_INSN(RT_VM_CONST, 4, 0, 0), 2,  /* fuzziness 0 */
        RT_VM_INSN(RT_VM_CONST, 5, 0, 0), 2,  /* transparency 0 */
        RT_VM_INSN(RT_VM_CONST, 6, 0, 0), 2,  /* refractive index 0 */
        RT_VM_INSN(RT_VM_CONST, 7, 0, 0), 3,  /* kd 1.0 */
        RT_VM_INSN(RT_VM_CONST, 8, 0, 0), 1,  /* ks 0.2 */
        RT_VM_INSN(RT_VM_CONST, 9, 0, 0), 3,  /* n 1.0 */
        RT_VM_INSN(RT_VM_RET, 0, 0, 0), 0,
    };
    const int32_t entry[1] = {0};
    rt_material dummy = mat(0, 0, 0, 0, 0, 0, 0, 0, 0, 0);
    rt_object objs[2];
    memset(objs, 0, sizeof objs);
    /* union(s at (-1.2, 0, 3), s at (1.2, 1, 3)) -> BFS order: the second first */
    const double pos[2][3] = {{1.2, 1.0, 3.0}, {-1.2, 0.0, 3.0}};
    for (int i = 0; i < 2; i++) {
        objs[i].kind = RT_SPHERE;
        objs[i].has_transform = 1;
        translate_uscale(objs[i].transform, pos[i][0], pos[i][1], pos[i][2], 1.0);
        for (int f = 0; f < RT_MAX_FACES; f++) objs[i].material[f] = -1; /* program 0 */
    }
    rt_point_light light = {{-10.0, 10.0, 0.0}, {1.0, 1.0, 1.0}};
    rt_scene sc;
    memset(&sc, 0, sizeof sc);
    sc.width = 1920;
    sc.height = 1200;
    sc.depth = 4;
    sc.fov = 90.0;
    sc.ambient[0] = sc.ambient[1] = sc.ambient[2] = 0.5;
    sc.num_lights = 1;
    sc.lights = &light;
    sc.objects = objs;
    sc.num_objects = 2;
    sc.materials = &dummy;
    sc.num_materials = 1;
    sc.program_code = code;
    sc.program_consts = consts;
    sc.program_entry = entry;
    sc.num_programs = 1;
    sc.program_code_words = (int32_t)(sizeof code / sizeof code[0]);
    sc.program_const_count = 4;
    return emit(&sc, out);
}

/* ---- file mode: a serialised rt_scene (go_raytracer_amd/scene.py write_scene_file) ---- */
static int rd(FILE *f, void *p, size_t n) { return n == 0 || fread(p, 1, n, f) == n; }

static void *rd_array(FILE *f, size_t elem, int32_t n, int *ok) {
    if (n <= 0) return NULL;
    void *p = malloc(elem * (size_t)n);
    if (!p || !rd(f, p, elem * (size_t)n)) *ok = 0;
    return p;
}

static int from_file(const char *scene_path, const char *out, const char *gather, int ndev, char **devs) {
    FILE *f = fopen(scene_path, "rb");
    if (!f) {
        fprintf(stderr, "cannot open %s\n", scene_path);
        return 2;
    }
    char magic[8];
    int32_t hdr[4], cnt[9];
    double dv[10];
    int ok = rd(f, magic, 8) && memcmp(magic, "RTSCENE1", 8) == 0 && rd(f, hdr, sizeof hdr) && rd(f, dv, sizeof dv) &&
             rd(f, cnt, sizeof cnt);
    rt_scene sc;
    memset(&sc, 0, sizeof sc);
    if (ok) {
        sc.width = hdr[0];
        sc.height = hdr[1];
        sc.depth = hdr[2];
        sc.num_lights = hdr[3];
        sc.fov = dv[0];
        for (int k = 0; k < 3; k++) {
            sc.ambient[k] = dv[1 + k];
            sc.bg_start[k] = dv[4 + k];
            sc.bg_end[k] = dv[7 + k];
        }
        sc.num_objects = cnt[0];
        sc.num_materials = cnt[1];
        sc.num_programs = cnt[2];
        sc.program_code_words = cnt[3];
        sc.program_const_count = cnt[4];
        sc.exp_mode = cnt[5];
        sc.num_ext_lights = cnt[6];
        sc.num_csg_leaves = cnt[7];
        sc.csg_code_words = cnt[8];
        sc.lights = rd_array(f, sizeof(rt_point_light), sc.num_lights, &ok);
        sc.objects = rd_array(f, sizeof(rt_object), sc.num_objects, &ok);
        sc.materials = rd_array(f, sizeof(rt_material), sc.num_materials, &ok);
        sc.program_code = rd_array(f, sizeof(uint32_t), sc.num_programs ? sc.program_code_words : 0, &ok);
        sc.program_consts = rd_array(f, sizeof(uint64_t), sc.num_programs ? sc.program_const_count : 0, &ok);
        sc.program_entry = rd_array(f, sizeof(int32_t), sc.num_programs, &ok);
        sc.ext_lights = rd_array(f, sizeof(rt_light), sc.num_ext_lights, &ok);
        sc.csg_leaves = rd_array(f, sizeof(rt_object), sc.num_csg_leaves, &ok);
        sc.csg_code = rd_array(f, sizeof(int32_t), sc.csg_code_words, &ok);
    }
    fclose(f);
    if (!ok) {
        fprintf(stderr, "malformed scene file %s\n", scene_path);
        return 2;
    }
    rt_render_opts o;
    memset(&o, 0, sizeof o);
    o.gather = !strcmp(gather, "peer") ? RT_GATHER_PEER : RT_GATHER_HOST;
    if (ndev > RT_MAX_DEVICES) return 2;
    if (ndev > 0) {
        o.device_count = ndev;
        o.flags = RT_RENDER_DEVICE_LIST;
        for (int i = 0; i < ndev; i++) o.devices[i] = atoi(devs[i]);
    }
    size_t bytes = (size_t)sc.width * sc.height * 4;
    uint8_t *pix = (uint8_t *)malloc(bytes);
    rt_stats st;
    if (!pix) return 2;
    int rc = rt_render_ex(&sc, &o, pix, &st);
    if (rc != RT_OK) {
        fprintf(stderr, "rt_render_ex failed (%d): %s\n", rc, rt_last_error());
        free(pix);
        return 1;
    }
    FILE *g = fopen(out, "wb");
    if (!g || fwrite(pix, 1, bytes, g) != bytes) {
        fprintf(stderr, "cannot write %s\n", out);
        free(pix);
        return 2;
    }
    fclose(g);
    free(pix);
    printf("{\"width\": %d, \"height\": %d, \"primary_rays\": %llu, \"secondary_rays\": %llu, \"shadow_rays\": %llu, "
           "\"shaded_hits\": %llu, \"surface_errors\": %llu, \"tests\": [",
           sc.width, sc.height, (unsigned long long)st.primary_rays, (unsigned long long)st.secondary_rays,
           (unsigned long long)st.shadow_rays, (unsigned long long)st.shaded_hits, (unsigned long long)st.surface_errors);
    for (int k = 0; k < RT_NUM_KINDS; k++) printf("%s%llu", k ? ", " : "", (unsigned long long)st.tests[k]);
    printf("], \"shadow_tests\": [");
    for (int k = 0; k < RT_NUM_KINDS; k++) printf("%s%llu", k ? ", " : "", (unsigned long long)st.shadow_tests[k]);
    printf("], \"devices\": %d, \"device_kernel_ms\": [", st.devices);
    for (int k = 0; k < st.devices; k++) printf("%s%.4f", k ? ", " : "", st.device_kernel_ms[k]);
    printf("], \"kernel_ms\": %.4f, \"gather_ms\": %.4f}\n", st.kernel_ms, st.gather_ms);
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 5 && !strcmp(argv[1], "file")) {
        if (rt_abi_version() != RT_ABI_VERSION) {
            fprintf(stderr, "ABI version mismatch\n");
            return 2;
        }
        return from_file(argv[2], argv[3], argv[4], argc - 5, argv + 5);
    }
    if (argc != 3) {
        fprintf(stderr, "usage: %s canned|sphere out.rgba | file scene.bin out.rgba host|peer [device ...]\n", argv[0]);
        return 2;
    }
    if (rt_abi_version() != RT_ABI_VERSION) {
        fprintf(stderr, "ABI version mismatch\n");
        return 2;
    }
    if (!strcmp(argv[1], "canned")) return canned(argv[2]);
    if (!strcmp(argv[1], "sphere")) return sphere(argv[2]);
    fprintf(stderr, "unknown scene %s\n", argv[1]);
    return 2;
}
