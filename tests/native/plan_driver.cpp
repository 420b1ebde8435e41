// Host planner driver for the sanitizer test (tests/test_sanitize_cpu.py):
// reads one image per stdin line
//   W H C target_w target_h flags gravity rotate smartcrop_w smartcrop_h
// and runs everything fi_plan.cpp builds for it -- plan_im, both tap axes,
// the k_rs_vm vertical tables and strips, the fused ring, the smartcrop plan
// with its Pillow tables and importance table -- printing a one-line digest.
// Built with -fsanitize=address,undefined (host only): any out-of-bounds
// access, overflow or UB in the planner aborts the run.
#include <stdio.h>

#include <vector>

#include "../../flyimg_amd/csrc/fi_plan.h"

using namespace fi;

int main() {
  int W, H, C, tw, th, rot, scw, sch, grav;
  unsigned flags;
  int n = 0, bad = 0;
  while (scanf("%d %d %d %d %d %u %d %d %d %d", &W, &H, &C, &tw, &th, &flags, &grav, &rot, &scw, &sch) == 10) {
    fi_image im{};
    im.src_w = W;
    im.src_h = H;
    im.src_channels = C;
    im.src_stride = W * C;
    im.target_w = tw;
    im.target_h = th;
    im.flags = flags;
    im.gravity = grav;
    im.rotate = rot;
    ImPlan p;
    const int rc = plan_im(im, &p);
    n++;
    if (rc != FI_OK) {
      printf("%d plan rc=%d %s\n", n, rc, p.err.c_str());
      continue;
    }
    long sum = 0;
    if (p.resize) {
      AxisTable v, h;
      build_axis(p.filter, p.yf, p.sh, p.th, p.ey0, p.ey0 + p.eh, p.sample, p.H, &v);
      build_axis(p.filter, p.xf, p.sw, p.tw, p.ex0, p.ex0 + p.ew, p.sample, p.W, &h);
      sum += v.touched + h.touched;
      VmV vm;
      if (build_vm_v(v, &vm)) sum += vm.nblk + (long)vm.frag.size();
      for (int mx : {64, 48, 32}) {
        MfmaH mh;
        if (build_mfma_h(h, &mh, mx)) sum += (long)mh.strips.size() + (long)mh.frag.size();
      }
      VrV vr;
      if (build_vr_v(v, &vr)) sum += vr.nblk + (long)vr.frag.size() + (long)vr.bmeta.size();
    }
    if (flags & FI_OP_SMARTCROP) {
      fi_smartcrop_options o{};
      o.prescale = 1;
      o.max_scale = 1;
      o.min_scale = 0.9;
      o.scale_step = 0.1;
      o.step = 8;
      o.exact_all = 1;
      ScPlan sp;
      const int src = plan_sc(p.out_w, p.out_h, scw > 0 ? scw : 100, sch > 0 ? sch : 100, o, &sp);
      if (src == FI_OK) {
        plan_sc_prep(&sp);
        fi_smartcrop_params prm{};
        prm.detail_weight = 0.2;
        prm.edge_radius = 0.4;
        prm.edge_weight = -10;
        prm.outside_importance = -0.5;
        prm.rule_of_thirds = 1;
        prm.score_down_sample = 1;
        std::vector<double> imp;
        if (!sp.crops.empty()) {
          const CropHost &c0 = sp.crops[0];
          sc_importance_table(prm, c0.fw, c0.fh, sp.aw, sp.ah, &imp);
        }
        sum += (long)sp.crops.size() + sp.aw + sp.ah + (long)imp.size();
      } else {
        printf("%d sc rc=%d\n", n, src);
      }
    }
    printf("%d ok %dx%dx%d %ld\n", n, p.out_w, p.out_h, p.out_c, sum);
  }
  printf("DONE %d images, %d bad\n", n, bad);
  return 0;
}
