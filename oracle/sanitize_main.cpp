// ORACLE — TEST INFRASTRUCTURE ONLY. ASan + UBSan driver of the CPU
// restatement (oracle/Makefile target `sanitize`, run by
// tests/test_oracle_sanitize.py). It pushes a short synthetic RGB-D sequence
// (and a stereo pair sequence) through every oracle entry the parity tests
// use: ORB extraction, LSD/LBD LineExtractor, the points+lines VO loop with
// and without the local map, and the stereo loop with lines, so that an
// out-of-bounds access or undefined arithmetic in the checker fails loudly
// instead of silently shaping the "expected" values.
//
// Input file (little-endian): int32 W, H, F, then F gray frames (u8 W*H),
// F depth frames (f32 W*H), F right frames (u8 W*H).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "oracle_api.h"

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s frames.bin\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int hdr[3];
  if (fread(hdr, 4, 3, f) != 3) return 2;
  const int W = hdr[0], H = hdr[1], F = hdr[2];
  const size_t px = (size_t)W * H;
  std::vector<uint8_t> gray(px * F), right(px * F);
  std::vector<float> depth(px * F);
  if (fread(gray.data(), 1, gray.size(), f) != gray.size()) return 2;
  if (fread(depth.data(), 4, depth.size(), f) != depth.size()) return 2;
  if (fread(right.data(), 1, right.size(), f) != right.size()) return 2;
  fclose(f);

  orbpl_orb_params orb{1000, 1.2f, 8, 20, 7};
  orbpl_camera cam{517.3f, 516.5f, 318.6f, 255.3f, 0.2624f, -0.9531f, -0.0054f, 0.0026f, 1.1633f,
                   40.0f, 40.0f * 40.0f / 517.3f, W, H};
  const int cap = 2 * orb.nfeatures + 64;
  std::vector<orbpl_keypoint> kps(cap);
  std::vector<uint8_t> desc((size_t)cap * 32);
  int n = 0;
  if (oracle_orb_extract(&orb, gray.data(), W, H, W, kps.data(), desc.data(), cap, &n, nullptr))
    return 1;
  std::vector<orbpl_keyline> kl(80);
  std::vector<uint8_t> ldesc(80 * 32);
  std::vector<double> coef(80 * 3);
  int nl = 0, nd = 0;
  if (oracle_line_extract(gray.data(), W, H, kl.data(), ldesc.data(), coef.data(), 80, &nl, &nd))
    return 1;
  printf("orb %d keypoints, lines %d of %d\n", n, nl, nd);

  // RGB-D points + lines, then with the local map and the analytic line Jacobian
  const int flag_sets[3] = {1, 1 | 4, 1 | 4 | 8};
  for (int fs : flag_sets) {
    void* v = oracle_lvo_create_ex(&orb, &cam, 1, fs);
    oracle_lvo_reset(v, nullptr);
    for (int k = 0; k < F; k++) {
      float T[16];
      int o[8];
      if (oracle_lvo_step(v, 0, gray.data() + px * k, depth.data() + px * k, T, o)) return 1;
      printf("flags %d frame %d: kps %d matches %d inliers %d lines %d line matches %d\n", fs, k,
             o[0], o[1], o[2], o[5], o[6]);
    }
    oracle_lvo_destroy(v);
  }
  // stereo with lines (rectified: no distortion)
  orbpl_camera scam = cam;
  scam.k1 = scam.k2 = scam.p1 = scam.p2 = scam.k3 = 0.0f;
  void* v = oracle_lvo_create_ex(&orb, &scam, 1, 1 | 2);
  oracle_lvo_reset(v, nullptr);
  for (int k = 0; k < F; k++) {
    float T[16];
    int o[8];
    if (oracle_lvo_step_stereo(v, 0, gray.data() + px * k, right.data() + px * k, T, o)) return 1;
    printf("stereo frame %d: kps %d matches %d lines %d line matches %d\n", k, o[0], o[1], o[5],
           o[6]);
  }
  oracle_lvo_destroy(v);
  printf("sanitize ok\n");
  return 0;
}
