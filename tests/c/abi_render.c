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

int main(int argc, char **argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s canned|sphere out.rgba\n", argv[0]);
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
