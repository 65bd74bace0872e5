// Host-side geometry of the ORB pipeline: the reference's constructor and
// per-level constants, evaluated once per configuration.
//   scale tables / features per level / umax : ORBextractor.cc:410-470
//   level sizes                               : ORBextractor.cc:1111-1113
//   FAST cell grid                            : ORBextractor.cc:769-806
//   DistributeOctTree initial nodes           : ORBextractor.cc:543-545
//   resize coefficient tables                 : OpenCV 3.4 hal::resize (8U, INTER_LINEAR)
#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/orbpl.h"
#include "orb_kernels.h"

namespace orbpl {

static int round_up(int v, int a) { return (v + a - 1) / a * a; }

int build_orb_geometry(int nfeatures, float scale_factor, int nlevels, int W, int H,
                       OrbHostGeom* out, const char** err) {
  *err = nullptr;
  if (nlevels < 1 || nlevels > kMaxLevels) { *err = "nlevels out of range [1,16]"; return ORBPL_ERR_ARG; }
  if (nfeatures < 1) { *err = "nfeatures must be >= 1"; return ORBPL_ERR_ARG; }
  if (!(scale_factor > 1.0f)) { *err = "scale_factor must be > 1"; return ORBPL_ERR_ARG; }
  if (W > 4000 || H > 4000) { *err = "image larger than 4000 px is not supported"; return ORBPL_ERR_ARG; }
  OrbHostGeom& G = *out;
  OrbGeom& g = G.g;
  g = OrbGeom{};
  g.nlevels = nlevels;
  g.W = W;
  g.H = H;
  // --- scale tables: float members, double scaleFactor (ORBextractor.h:80) ---
  const double sf = (double)scale_factor;
  G.scale.assign(nlevels, 1.0f);
  G.sigma2.assign(nlevels, 1.0f);
  for (int i = 1; i < nlevels; i++) {
    G.scale[i] = (float)(G.scale[i - 1] * sf);
    G.sigma2[i] = G.scale[i] * G.scale[i];
  }
  G.inv_scale.resize(nlevels);
  G.inv_sigma2.resize(nlevels);
  for (int i = 0; i < nlevels; i++) {
    G.inv_scale[i] = 1.0f / G.scale[i];
    G.inv_sigma2[i] = 1.0f / G.sigma2[i];
  }
  std::vector<int> nfeat(nlevels);
  {
    const float factor = (float)(1.0f / sf);
    float nd = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
      nfeat[l] = (int)std::rint(nd);
      sum += nfeat[l];
      nd *= factor;
    }
    nfeat[nlevels - 1] = std::max(nfeatures - sum, 0);
  }
  // --- umax (IC_Angle patch) ---
  {
    const int HP = 15;
    int v, v0;
    const int vmax = (int)std::floor(HP * std::sqrt(2.f) / 2 + 1);
    const int vmin = (int)std::ceil(HP * std::sqrt(2.f) / 2);
    const double hp2 = HP * HP;
    for (v = 0; v <= vmax; ++v) g.umax[v] = (int)std::rint(std::sqrt(hp2 - v * v));
    for (v = HP, v0 = 0; v >= vmin; --v) {
      while (g.umax[v0] == g.umax[v0 + 1]) ++v0;
      g.umax[v] = v0;
      ++v0;
    }
  }
  // --- levels ---
  long long off = 0, boff = 0;
  int cell_total = 0, kp_total = 0;
  int max_slots = 1;
  G.cells.clear();
  G.rs.clear();
  std::vector<std::vector<CellGeom>> lvl_cells(nlevels);
  for (int l = 0; l < nlevels; l++) {
    LevelGeom& L = g.lv[l];
    L.w = (int)std::rint((float)W * G.inv_scale[l]);
    L.h = (int)std::rint((float)H * G.inv_scale[l]);
    if (L.w < 20 || L.h < 20) {
      *err = "a pyramid level is smaller than 20 px (image too small for nlevels/scale)";
      return ORBPL_ERR_ARG;
    }
    L.pw = L.w + 2 * kEdge;
    L.ph = L.h + 2 * kEdge;
    L.pitch = round_up(kLead + L.pw, 16);
    L.pyr_off = off;
    off += (long long)round_up(L.pitch * L.ph, 256);
    L.bpitch = round_up(L.w, 16);
    L.boff = boff;
    boff += (long long)round_up(L.bpitch * L.h, 256);
    L.scale = G.scale[l];
    L.nfeat = nfeat[l];
    L.scaled_patch = (int)(31 * G.scale[l]);
    // FAST cells
    const int minB = kMinBorder;
    const int maxBX = L.w - kEdge + 3, maxBY = L.h - kEdge + 3;
    L.max_border_x = maxBX;
    L.max_border_y = maxBY;
    const float width = (float)(maxBX - minB), height = (float)(maxBY - minB);
    const int nCols = (int)(width / 30.f), nRows = (int)(height / 30.f);
    L.ncols = nCols;
    L.nrows = nRows;
    L.wcell = nCols > 0 ? (int)std::ceil(width / nCols) : 0;
    L.hcell = nRows > 0 ? (int)std::ceil(height / nRows) : 0;
    L.ncells = nCols * nRows;
    L.cell_base = cell_total;
    for (int i = 0; i < nRows; i++) {
      const float iniY = (float)(minB + i * L.hcell);
      float maxY = iniY + L.hcell + 6;
      for (int j = 0; j < nCols; j++) {
        CellGeom c{};
        c.level = (int16_t)l;
        const float iniX = (float)(minB + j * L.wcell);
        float maxX = iniX + L.wcell + 6;
        bool skip = (iniY >= maxBY - 3) || (iniX >= maxBX - 6);
        if (!skip) {
          float my = maxY > maxBY ? (float)maxBY : maxY;
          float mx = maxX > maxBX ? (float)maxBX : maxX;
          c.x0 = (int16_t)iniX;
          c.y0 = (int16_t)iniY;
          c.x1 = (int16_t)mx;
          c.y1 = (int16_t)my;
          g.fast_win_w = std::max(g.fast_win_w, c.x1 - c.x0);
          g.fast_win_h = std::max(g.fast_win_h, c.y1 - c.y0);
          const int dw = c.x1 - c.x0 - 6, dh = c.y1 - c.y0 - 6;
          if (dw > 0 && dh > 0) max_slots = std::max(max_slots, ((dw + 1) / 2) * ((dh + 1) / 2));
          if (c.x1 - c.x0 > 66 || c.y1 - c.y0 > 66) {
            *err = "FAST window larger than 66 px";
            return ORBPL_ERR_ARG;
          }
        }
        lvl_cells[l].push_back(c);
      }
    }
    if (L.ncells > 1024) { *err = "more than 1024 FAST cells in one level"; return ORBPL_ERR_ARG; }
    cell_total += L.ncells;
    // octree initial nodes (pinned: nIni >= 1)
    int nIni = (int)std::round((float)(maxBX - minB) / (float)(maxBY - minB));
    if (nIni < 1) nIni = 1;
    L.n_ini = nIni;
    L.hx = (float)(maxBX - minB) / nIni;
    L.kp_cap = std::max(L.nfeat + 3, 4 * nIni);
    if (L.kp_cap > kOctMaxList || nIni > kOctMaxList) {
      *err = "features per level exceed the octree list capacity (1024)";
      return ORBPL_ERR_ARG;
    }
    L.kp_base = kp_total;
    kp_total += L.kp_cap;
  }
  for (int l = 0; l < nlevels; l++) G.cells.insert(G.cells.end(), lvl_cells[l].begin(), lvl_cells[l].end());
  g.ncells_total = cell_total;
  g.kp_cap_total = kp_total;
  g.cell_slots = max_slots;
  g.pyr_bytes = off;
  g.blur_bytes = boff;
  int cand_total = 0;
  for (int l = 0; l < nlevels; l++) {
    LevelGeom& L = g.lv[l];
    L.cand_base = cand_total;
    L.cand_cap = L.ncells * max_slots;
    if (L.cand_cap > kMaxCandPerLevel) { *err = "candidate capacity per level exceeds 2^20"; return ORBPL_ERR_ARG; }
    cand_total += L.cand_cap;
  }
  g.cand_cap_total = cand_total;
  // --- resize tables (OpenCV hal::resize, INTER_LINEAR, 8U fixed point) ---
  for (int l = 1; l < nlevels; l++) {
    LevelGeom& L = g.lv[l];
    const LevelGeom& S = g.lv[l - 1];
    L.rs_off = (int)G.rs.size();
    const int sw = S.w, sh = S.h, dw = L.w, dh = L.h;
    const double isx = (double)dw / sw, isy = (double)dh / sh;
    const double scx = 1. / isx, scy = 1. / isy;
    std::vector<int> xofs(dw), alpha(dw), yofs(dh), beta(dh);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
      float fx = (float)((dx + 0.5) * scx - 0.5);
      int sx = (int)std::floor(fx);
      fx -= sx;
      if (sx < 0) { fx = 0; sx = 0; }
      if (sx + 1 >= sw) {
        xmax = std::min(xmax, dx);
        if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
      }
      xofs[dx] = sx;
      int a0 = (int)std::rint((1.f - fx) * 2048.f), a1 = (int)std::rint(fx * 2048.f);
      alpha[dx] = (a0 & 0xFFFF) | (a1 << 16);
    }
    for (int dy = 0; dy < dh; dy++) {
      float fy = (float)((dy + 0.5) * scy - 0.5);
      int sy = (int)std::floor(fy);
      fy -= sy;
      yofs[dy] = sy;
      int b0 = (int)std::rint((1.f - fy) * 2048.f), b1 = (int)std::rint(fy * 2048.f);
      beta[dy] = (b0 & 0xFFFF) | (b1 << 16);
    }
    L.xmax = xmax;
    // k_pyramid resize walk: the source bytes of 4 adjacent output columns
    // (xofs .. xofs + 1) must lie in 3 dwords from xofs[x] & ~3
    for (int x = 0; x < dw; x += 4) {
      const int x3 = std::min(x + 3, dw - 1);
      if (xofs[x3] + 1 - (xofs[x] & ~3) > 11) {
        *err = "scale factor too large for the resize walk";
        return ORBPL_ERR_ARG;
      }
    }
    G.rs.insert(G.rs.end(), xofs.begin(), xofs.end());
    G.rs.insert(G.rs.end(), alpha.begin(), alpha.end());
    G.rs.insert(G.rs.end(), yofs.begin(), yofs.end());
    G.rs.insert(G.rs.end(), beta.begin(), beta.end());
  }
  if (G.rs.empty()) G.rs.push_back(0);
  // --- k_pyramid row bands for B = 1, 2, 4, 8 ---
  // own rows partition each level; need rows = own +- 3 (blur) united with
  // the source rows (yofs, yofs + 1, clamped) of the next level's need rows
  G.bands.assign(2 * kPyrMaxBands - 1, PyrBand{});
  for (int B = 1; B <= kPyrMaxBands; B *= 2) {
    for (int b = 0; b < B; b++) {
      PyrBand& P = G.bands[pyr_band_base(B) + b];
      for (int l = nlevels - 1; l >= 0; l--) {
        const int h = g.lv[l].h;
        P.oa[l] = (int)((long long)b * h / B);
        P.ob[l] = (int)((long long)(b + 1) * h / B);
        int na = std::max(0, P.oa[l] - 3), nb = std::min(h, P.ob[l] + 3);
        if (l + 1 < nlevels) {
          const LevelGeom& U = g.lv[l + 1];
          const int* yofs = G.rs.data() + U.rs_off + 2 * U.w;
          na = std::min(na, std::min(std::max(yofs[P.na[l + 1]], 0), h - 1));
          nb = std::max(nb, std::min(std::max(yofs[P.nb[l + 1] - 1] + 1, 0), h - 1) + 1);
        }
        P.na[l] = na;
        P.nb[l] = nb;
      }
    }
  }
  return ORBPL_OK;
}

}  // namespace orbpl
