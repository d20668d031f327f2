// Host-side sanitizer harness (SURVEY §5 "race detection / sanitizers"): the kernels' host code -- tile cost
// models, grid sizing, shape validation -- compiled with AddressSanitizer + UBSan (host only: GPU sanitizers are
// not available on this pool) and swept over every encoder / transformer shape family.  No GPU needed: nothing
// here launches; invalid shapes must be rejected before any launch.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../../pytorch_rt1_for_distributed_training_amd/csrc/rt1_kernels.h"

static int failures = 0;
#define EXPECT(c)                                                                   \
    do {                                                                            \
        if (!(c)) {                                                                 \
            std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);     \
            ++failures;                                                             \
        }                                                                           \
    } while (0)

int main() {
    // depthwise grids: every (resolution, channel, kernel, stride) family of B3 at three input sizes
    const int res[] = {150, 128, 75, 64, 38, 32, 19, 16, 10, 8, 5, 1};
    const int chans[] = {40, 24, 144, 192, 288, 336, 576, 672, 816, 1152, 1392, 2304, 8, 16};
    const int frames[] = {1, 7, 48, 768};
    long checked = 0;
    for (int n : frames)
        for (int h : res)
            for (int c : chans)
                for (int k = 3; k <= 5; k += 2)
                    for (int s = 1; s <= 2; ++s)
                        for (int flag = 0; flag < 2; ++flag) {
                            const int w = h + 7 * (h % 3);
                            const int g1 = rt1_dw_grid(n, h, w, c, k, s, 4096, flag, 1 - flag);
                            const int g2 = rt1_dw_wgrad_grid(n, h, w, c, k, s, 1024, flag);
                            const int g3 = rt1_dw_bwd_grid(n, h, w, c, k, s, 4096, flag);
                            if (s == 2) EXPECT(rt1_dw_bwd_fused_s2_grid(n, h, w, c, k, 4096, flag, 0) >= 1);
                            else EXPECT(rt1_dw_bwd_fused_grid(n, h, w, c, k, 4096, flag, flag, -1, 0) >= 1);
                            // x-mode tile search (y1-free expand blocks) for the shapes that have a specialisation
                            for (int cin : {24, 32, 48}) {
                                if (!rt1_dw_x_supported(cin, c, k, s)) continue;
                                int info[4];
                                EXPECT(rt1_dw_grid_x(n, h, w, c, k, s, cin, 4096) >= 1);
                                EXPECT(rt1_dw_tile_info(1, h, w, c, k, s, cin, info) == 0 && info[0] >= 1 &&
                                       info[1] >= 1 && info[2] <= 160 * 1024);
                                if (s == 2) EXPECT(rt1_dw_bwd_fused_s2_grid(n, h, w, c, k, 4096, 1, cin) >= 1);
                                else EXPECT(rt1_dw_bwd_fused_grid(n, h, w, c, k, 4096, 1, 1, 1, cin) >= 1);
                            }
                            EXPECT(g1 >= 1 && g1 <= 4096);
                            EXPECT(g2 >= 1 && g2 <= 1024);
                            EXPECT(g3 >= 1 && g3 <= 4096);
                            ++checked;
                        }
    // pointwise GEMM dispatch tables
    for (int K = 8; K <= 2560; K += 8)
        for (int N = 8; N <= 2560; N += 8) {
            if (rt1_pw_gemm_supported(K, N)) {
                const int g = rt1_pw_gemm_grid(1 << 20, K, N, 2048);
                EXPECT(g >= 1 && g <= 2048);
            }
            if (rt1_pw_tall_preferred(K, N)) EXPECT(rt1_pw_tall_supported(K, N));
            if (rt1_pw_tall_supported(K, N)) EXPECT(K > N && N <= 384 && K % 8 == 0);
            rt1_pw_wide_supported(K, N);
            ++checked;
        }
    // unsupported shapes are rejected before any launch (no device, no stream needed)
    EXPECT(rt1_pw_tall(nullptr, nullptr, 1000, 96, 576, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr) != 0);
    EXPECT(rt1_pw_tall(nullptr, nullptr, 0, 576, 96, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr) != 0);
    // the operand prologue needs shift + gate and whole frames (M % hw == 0)
    float dummy = 0.f;
    EXPECT(rt1_pw_tall(nullptr, nullptr, 1000, 576, 96, nullptr, &dummy, &dummy, nullptr, 361, nullptr, nullptr) != 0);
    EXPECT(rt1_pw_tall(nullptr, nullptr, 1000, 576, 96, nullptr, &dummy, &dummy, &dummy, 361, nullptr, nullptr) != 0);  // 1000 % 361
    EXPECT(rt1_embed_fwd(nullptr, nullptr, nullptr, nullptr, 100, 510, 512, 66, nullptr, nullptr) != 0);
    EXPECT(rt1_embed_fwd(nullptr, nullptr, nullptr, nullptr, 100, 512, 500, 66, nullptr, nullptr) != 0);
    for (int ce = 8; ce <= 512; ce += 8)
        for (int ci = 8; ci <= 128; ci += 8) rt1_pw_bwd_supported(ce, ci);
    for (int m : {1, 1000, 1 << 22}) EXPECT(rt1_pw_bwd_grid(m, 512) >= 1);
    for (int n : frames)
        for (int hw : {22500, 5700, 1444, 361, 100, 1})
            for (int c : chans) {
                const int s = rt1_frame_splits(n, hw, c);
                EXPECT(s >= 1);
            }
    for (int n : frames)
        for (int h : {300, 256, 456, 128, 16}) EXPECT(rt1_stem_grid(n, h, h + 40, 8192) >= 1);
    for (int t : {1, 66, 165, 8448, 1 << 20}) EXPECT(rt1_tf_grid(t) >= 1);
    for (int p : {1, 64, 100, 120, 225, 256, 257, 1000}) rt1_tl_supported(p, 512, 64, 8);
    EXPECT(!rt1_tl_supported(257, 512, 64, 8));
    for (int v : {2, 128, 256, 512, 1024, 4096}) rt1_head_ce_supported(v, 512);
    std::printf("host checks: %ld shape cases, %d failures\n", checked, failures);
    return failures == 0 ? 0 : 1;
}
