// Host cost of the per-geometry resample tables (fi_plan.cpp) on cfg4-like
// geometries: build_axis (both axes), build_vm_v, build_mfma_h.
//   hipcc -O2 -std=c++17 -I include tools/plan_bench.cpp flyimg_amd/csrc/fi_plan.cpp -o /tmp/plan_bench
#include <chrono>
#include <cmath>
#include <cstdio>
#include <random>

#include "../flyimg_amd/csrc/fi_plan.h"

using namespace fi;

int main() {
  std::mt19937_64 rng(20250112);
  std::uniform_real_distribution<double> U(std::log(0.5), std::log(24.0));
  const double aspects[6] = {4.0 / 3, 1.5, 16.0 / 9, 1.0, 2.0 / 3, 9.0 / 16};
  const char *ops[5] = {"w_300,h_250,c_1", "w_500,smc_1", "w_512,h_512,c_1", "h_300", "w_400,h_400,c_1"};
  double t_axis = 0, t_v = 0, t_h = 0;
  size_t vbytes = 0, hbytes = 0;
  const int n = 200;
  for (int i = 0; i < n; i++) {
    const double mp = std::exp(U(rng));
    const double a = aspects[rng() % 6];
    const int W = std::max(16, (int)std::lround(std::sqrt(mp * 1e6 * a))), H = std::max(16, (int)std::lround(W / a));
    fi_image img{};
    img.src_w = W;
    img.src_h = H;
    img.src_stride = W * 3;
    img.src_channels = 3;
    img.flags = FI_OP_THUMBNAIL;
    const int k = i % 5;
    if (k == 0) { img.target_w = 300; img.target_h = 250; img.flags |= FI_GEOM_FILL | FI_OP_EXTENT; }
    if (k == 1) { img.target_w = 500; img.flags |= FI_GEOM_SHRINK_ONLY; }
    if (k == 2) { img.target_w = 512; img.target_h = 512; img.flags |= FI_GEOM_FILL | FI_OP_EXTENT; }
    if (k == 3) { img.target_h = 300; img.flags |= FI_GEOM_SHRINK_ONLY; }
    if (k == 4) { img.target_w = 400; img.target_h = 400; img.flags |= FI_GEOM_FILL | FI_OP_EXTENT; }
    ImPlan P;
    if (plan_im(img, &P) != FI_OK || !P.resize) continue;
    auto t0 = std::chrono::steady_clock::now();
    AxisTable vt, ht;
    build_axis(P.filter, P.yf, P.sh, P.th, P.ey0, P.ey0 + P.eh, P.sample, P.H, &vt);
    build_axis(P.filter, P.xf, P.sw, P.tw, P.ex0, P.ex0 + P.ew, P.sample, P.W, &ht);
    auto t1 = std::chrono::steady_clock::now();
    VmV vv;
    build_vm_v(vt, &vv);
    auto t2 = std::chrono::steady_clock::now();
    MfmaH mh;
    build_mfma_h(ht, &mh, 64);
    auto t3 = std::chrono::steady_clock::now();
    t_axis += std::chrono::duration<double, std::milli>(t1 - t0).count();
    t_v += std::chrono::duration<double, std::milli>(t2 - t1).count();
    t_h += std::chrono::duration<double, std::milli>(t3 - t2).count();
    vbytes += vv.frag.size() * 4;
    hbytes += mh.frag.size() * 4;
    (void)ops;
  }
  printf("per geometry: axis %.3f ms, vm_v %.3f ms (%.0f KB frag), mfma_h %.3f ms (%.0f KB frag)\n", t_axis / n,
         t_v / n, vbytes / 1024.0 / n, t_h / n, hbytes / 1024.0 / n);
}
