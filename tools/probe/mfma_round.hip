// Probe: rounding of v_mfma_f32_16x16x32_bf16 (C + Σ a·b) on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const float* av, const float* bv, const float* cv, float* out) {
    const int l = threadIdx.x;
    bf16x8 a, b;
    for (int e = 0; e < 8; ++e) { a[e] = (__bf16)av[l * 8 + e]; b[e] = (__bf16)bv[l * 8 + e]; }
    f32x4 c = {cv[l * 4], cv[l * 4 + 1], cv[l * 4 + 2], cv[l * 4 + 3]};
    f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[l * 4 + r] = d[r];
}
// case: products placed at (row 0, col 0): A[0][k], B[k][0]; lane l holds A[l&15][8(l>>4)+e], B[8(l>>4)+e][l&15]
int main() {
    float *a, *b, *c, *o;
    hipMalloc(&a, 512 * 4); hipMalloc(&b, 512 * 4); hipMalloc(&c, 256 * 4); hipMalloc(&o, 256 * 4);
    struct Case { const char* name; float cval; int n; float pa[4], pb[4]; };
    const float u = 1.0f / (1 << 12);
    Case cases[] = {
        {"C=1 + 0.75ulp (one product)", 1.f, 1, {1.5f * u}, {u}},
        {"C=-1 - 0.75ulp", -1.f, 1, {-1.5f * u}, {u}},
        {"C=1 + 0.25ulp", 1.f, 1, {0.5f * u}, {u}},
        {"C=0: 1 + 0.75ulp (two products)", 0.f, 2, {1.f, 1.5f * u}, {1.f, u}},
        {"C=0: -1 - 0.75ulp (two products)", 0.f, 2, {-1.f, -1.5f * u}, {1.f, u}},
        {"C=1 + 0.5ulp tie (even stays)", 1.f, 1, {1.f * u}, {u}},
        {"C=1+ulp + 0.5ulp tie (odd rounds up)", 1.0000001192092896f, 1, {1.f * u}, {u}},
        {"C=0: 1 + 0.375ulp + 0.375ulp", 0.f, 3, {1.f, 0.75f * u, 0.75f * u}, {1.f, u, u}},
    };
    for (const Case& cs : cases) {
        float ha[512] = {0}, hb[512] = {0}, hc[256] = {0}, ho[256];
        for (int i = 0; i < cs.n; ++i) {
            // k = i: lane (k/8)*16 + row0 holds A[0][k] at e = k%8; B[k][0] in lane (k/8)*16 + 0
            const int lane = (i / 8) * 16, e = i % 8;
            ha[lane * 8 + e] = cs.pa[i];
            hb[lane * 8 + e] = cs.pb[i];
        }
        hc[0] = cs.cval;  // D[row 0][col 0] = lane 0, reg 0
        hipMemcpy(a, ha, sizeof ha, hipMemcpyHostToDevice);
        hipMemcpy(b, hb, sizeof hb, hipMemcpyHostToDevice);
        hipMemcpy(c, hc, sizeof hc, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, a, b, c, o);
        hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
        double exact = cs.cval;
        for (int i = 0; i < cs.n; ++i) exact += (double)cs.pa[i] * cs.pb[i];
        printf("%-40s D=%.10g (bits %08x)  exact=%.12g  fp32-RNE=%.10g\n", cs.name, ho[0],
               *(unsigned*)&ho[0], exact, (float)exact);
    }
    return 0;
}
