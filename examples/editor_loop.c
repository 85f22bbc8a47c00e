/*
 * editor_loop.c — a native host of the C ABI (include/wcpt.h) that drives the path the way the reference's Jai
 * editor does, with nothing but plain C. It is what the Jai #foreign glue of INTEGRATION.md does, written out:
 *
 *   Init (PathTracingRenderer.jai:272-343)      scene + OBJ path -> BVH -> six device buffers + DrawCommand
 *   CreateScreen (:345-385)                      rgba32f image
 *   per frame (editor.jai:149-158)               camera still ? renderedFramesCount += 1 : = 0
 *                                                UpdateMaterials (:459-471) -> Render (:399-457, count += 1)
 *   display (composite.comp)                     gamma + PBR Neutral -> RGBA8 -> PPM file
 *
 *   usage: editor_loop [scene=cornell] [width=640] [height=360] [frames=8] [out.ppm] [--move-at K]
 *
 * Prints one line per frame with the renderedFramesCount the dispatch used and the frame time. Exit code 0 on
 * success; any wcpt error is printed with wcpt_last_error and returned as the exit code's magnitude.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/wcpt.h"

#define CHECK(ctx, call)                                                                      \
    do {                                                                                      \
        int rc_ = (call);                                                                     \
        if (rc_ != WCPT_SUCCESS) {                                                            \
            fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, wcpt_last_error(ctx));       \
            return rc_ < 0 ? -rc_ : rc_;                                                      \
        }                                                                                     \
    } while (0)

static double now_ms(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

/* DBufferManager.Update (BufferManager.jai:52-64): allocate on first use, upload (grows), return the address */
static int upload(wcpt_context* ctx, wcpt_buffer* buf, const void* data, uint64_t bytes, uint64_t* addr)
{
    int rc;
    if (*buf == 0 && (rc = wcpt_buffer_alloc(ctx, bytes, buf)) != WCPT_SUCCESS) return rc;
    if ((rc = wcpt_buffer_upload(ctx, *buf, data, bytes, 0)) != WCPT_SUCCESS) return rc;
    *addr = wcpt_buffer_device_address(ctx, *buf);
    return *addr ? WCPT_SUCCESS : WCPT_ERROR_INVALID_HANDLE;
}

int main(int argc, char** argv)
{
    const char* scene_name = argc > 1 ? argv[1] : "cornell";
    const uint32_t W = argc > 2 ? (uint32_t)atoi(argv[2]) : 640;
    const uint32_t H = argc > 3 ? (uint32_t)atoi(argv[3]) : 360;
    const int frames = argc > 4 ? atoi(argv[4]) : 8;
    const char* out_path = argc > 5 ? argv[5] : "editor_loop.ppm";
    int move_at = -1;
    for (int i = 1; i + 1 < argc; i++)
        if (strcmp(argv[i], "--move-at") == 0) move_at = atoi(argv[i + 1]);

    /* ---- Init: scene, mesh -> BVH (LoadModel :219-270) ------------------------------------------------ */
    wcpt_scene sc;
    if (wcpt_scene_generate(scene_name, 0, &sc) != WCPT_SUCCESS) {
        fprintf(stderr, "scene '%s': %s\n", scene_name, wcpt_last_error(NULL));
        return 2;
    }
    const uint32_t max_nodes = sc.mesh.index_count ? 2u * sc.mesh.index_count / 3u + 1u : 1u;
    wcpt_node* nodes = (wcpt_node*)calloc(max_nodes, sizeof(wcpt_node));
    uint32_t node_count = 0;
    if (sc.mesh.index_count &&
        wcpt_bvh_build(sc.mesh.positions, sc.mesh.vertex_count, sc.mesh.indices, sc.mesh.index_count, nodes,
                       max_nodes, &node_count) != WCPT_SUCCESS) {
        fprintf(stderr, "bvh: %s\n", wcpt_last_error(NULL));
        return 2;
    }

    wcpt_context* ctx = NULL;
    CHECK(NULL, wcpt_create(0, &ctx));
    wcpt_buffer b_vtx = 0, b_idx = 0, b_bvh = 0, b_draw = 0, b_mat = 0, b_sph = 0, b_out = 0;
    uint64_t a_vtx = 0, a_idx = 0, a_bvh = 0, a_draw = 0, a_mat = 0, a_sph = 0;
    uint32_t draw_count = 0;
    if (sc.mesh.index_count) {
        CHECK(ctx, upload(ctx, &b_vtx, sc.mesh.positions, (uint64_t)sc.mesh.vertex_count * 12u, &a_vtx));
        CHECK(ctx, upload(ctx, &b_idx, sc.mesh.indices, (uint64_t)sc.mesh.index_count * 4u, &a_idx));
        CHECK(ctx, upload(ctx, &b_bvh, nodes, (uint64_t)node_count * sizeof(wcpt_node), &a_bvh));
        wcpt_draw_command dc;
        memset(&dc, 0, sizeof(dc));
        dc.vertexBuffer = a_vtx;                /* GetDeviceAddress (PathTracingRenderer.jai:251-256) */
        dc.indexBuffer = a_idx;
        dc.bvhBuffer = a_bvh;
        dc.indexCount = sc.mesh.index_count;
        CHECK(ctx, upload(ctx, &b_draw, &dc, sizeof(dc), &a_draw));
        draw_count = 1;
    }

    /* ---- CreateScreen ------------------------------------------------------------------------------------ */
    CHECK(ctx, wcpt_create_screen(ctx, W, H));
    CHECK(ctx, wcpt_buffer_alloc(ctx, (uint64_t)W * H * 4u, &b_out));

    /* ---- frames: editor.jai:149-158 --------------------------------------------------------------------- */
    uint32_t renderedFramesCount = 0;
    wcpt_camera cam = sc.camera;
    for (int f = 0; f < frames; f++) {
        const int moved = (f == move_at);
        if (moved) {
            cam.yaw += 1.0f;
            renderedFramesCount = 0;
        } else {
            renderedFramesCount += 1;
        }
        CHECK(ctx, wcpt_camera_update(&cam, (float)W / (float)H));          /* Update(*camera, aspect) */
        CHECK(ctx, upload(ctx, &b_mat, sc.materials, (uint64_t)sc.material_count * sizeof(wcpt_material), &a_mat));
        CHECK(ctx, upload(ctx, &b_sph, sc.spheres, (uint64_t)sc.sphere_count * sizeof(wcpt_sphere), &a_sph));
        wcpt_scene_data sd;                                                  /* Render :410-422 */
        memset(&sd, 0, sizeof(sd));
        memcpy(sd.inverseProjection, cam.inverseProjection, sizeof(sd.inverseProjection));
        memcpy(sd.inverseView, cam.inverseView, sizeof(sd.inverseView));
        memcpy(sd.position, cam.position, sizeof(sd.position));
        sd.maxBounceCount = 3;
        sd.samples = 1;
        sd.sphereCount = sc.sphere_count;
        sd.drawCommandCount = draw_count;
        sd.renderedFramesCount = renderedFramesCount;
        const double t0 = now_ms();
        CHECK(ctx, wcpt_render(ctx, &sd, a_mat, a_sph, a_draw));
        CHECK(ctx, wcpt_sync(ctx));
        const double t1 = now_ms();
        renderedFramesCount += 1;                                            /* :423 */
        printf("frame %d renderedFramesCount %u %s %.3f ms\n", f, sd.renderedFramesCount, moved ? "(moved)" : "",
               t1 - t0);
    }

    /* ---- display: composite.comp -> RGBA8 -> PPM ---------------------------------------------------------- */
    CHECK(ctx, wcpt_composite(ctx, wcpt_buffer_device_address(ctx, b_out), WCPT_COMPOSITE_RGBA8));
    CHECK(ctx, wcpt_sync(ctx));
    uint8_t* px = (uint8_t*)malloc((size_t)W * H * 4u);
    CHECK(ctx, wcpt_buffer_download(ctx, b_out, px, (uint64_t)W * H * 4u, 0));
    FILE* fp = fopen(out_path, "wb");
    if (fp) {
        fprintf(fp, "P6\n%u %u\n255\n", W, H);
        for (uint64_t i = 0; i < (uint64_t)W * H; i++) fwrite(px + 4 * i, 1, 3, fp);
        fclose(fp);
        printf("wrote %s\n", out_path);
    }

    /* ---- Deinit (:473-490) -------------------------------------------------------------------------------- */
    free(px);
    free(nodes);
    wcpt_buffer bufs[] = {b_vtx, b_idx, b_bvh, b_draw, b_mat, b_sph, b_out};
    for (size_t i = 0; i < sizeof(bufs) / sizeof(bufs[0]); i++)
        if (bufs[i]) wcpt_buffer_free(ctx, bufs[i]);
    wcpt_destroy(ctx);
    wcpt_scene_free(&sc);
    return 0;
}
