// CPU model of a round-free speculative LSD seed loop (development tool, not
// product code): one wave of 64 lanes in lockstep emulated on the host, over
// the oracle's LSD restatement (oracle/lsd_oracle.cpp, included as text so
// the restatement's numerics are used unchanged).
//
// Schedule modelled ("streaming"):
//   * seeds are fetched in list order into a reorder window; the claim tag of
//     a seed is its fetch index (smaller = earlier), the stamp of a pixel is
//     0 (USED, committed), 0xFFFFFFFF (free) or tag << 1 | gen;
//   * every lane grows its own seed one point expansion per iteration; a lane
//     whose region is done takes the next seed at once (no round barrier);
//     an aligned, uncommitted neighbour claimed by an earlier in-flight seed
//     aborts the grow (conflict, the seed is redone when it is the head);
//   * regions reaching min_reg_size wait for a fit batch (region2rect, refine
//     with its second grow, reduce_region_radius);
//   * seeds commit in fetch order from the head: the touched pixels must
//     still carry the seed's own tag, the final region becomes USED, the
//     other touched pixels are released; a conflicting head seed whose seed
//     pixel is now USED is skipped, otherwise regrown by the next free lane
//     (exact: every earlier seed is committed).
// The candidate rectangles must equal the sequential loop's (checked), and
// the model reports lockstep iterations and a cycle estimate next to the
// round-synchronous schedule of k_lsd_spec (rounds of 64 seeds, each costing
// its slowest lane) under the same cost constants.
//
// build + run: python tools/lsd_stream_sim.py [frames] [window] [fit_batch]
//
// Measured on MI355X in round 5 (k_lsd_stream, git history 5591b98..3bef507;
// bit-exact: the 26 LSD parity tests passed with it at every step): at batch 1
// 104-139M shader cycles per frame against the round loop's 99-105M on the
// same boxes (profiles/r05/lsd_stream_ab.txt). Each lockstep iteration's
// bookkeeping (seed queue, releases, refetches, the in-order commit's two
// dependent loads per seed) and the lanes parked behind fit batches outweigh
// the removed round barrier; a larger window (1024 slots) fetched 31.8k
// instead of 27k seeds and ran slower still. Not kept.
#include "../oracle/lsd_oracle.cpp"

#include <cstdio>
#include <deque>

namespace lsdo {

struct Cost {
  // cycles, calibrated on round 4's per-frame split of k_lsd_spec at batch 1
  // (first grows 43.5M, fits 48.1M, re-check + commit 7.4M, scans 3.2M over
  // 388 rounds)
  double step = 4000;         // one lockstep grow step (a dependent neighbourhood round trip)
  double fit_fixed = 25000;   // a fit batch's fixed passes (group setup, barriers)
  double pass64 = 2500;       // one wave-wide pass over 64 list entries of a group
  double commit_seed = 250;   // commit / check of one seed (uniform control)
  double commit_px = 60;      // per touched pixel re-read / released (one lane)
  double scan64 = 400;        // scanning 64 list entries for seeds
};

constexpr uint32_t kFree = 0xFFFFFFFFu;

struct Sim {
  LSD& L;
  int W, H;
  double prec, p;
  size_t min_reg;
  std::vector<uint32_t> stamp;

  explicit Sim(LSD& l, double prec_, double p_, size_t mr)
      : L(l), W(l.img_width), H(l.img_height), prec(prec_), p(p_), min_reg(mr) {
    stamp.assign((size_t)W * H, kFree);
  }

  // a resumable region grow (region_grow, lsd.cpp) over stamps
  struct Grow {
    std::vector<RegionPoint> reg;
    size_t i = 0;
    double reg_angle = 0;
    float sumdx = 0, sumdy = 0;
    double prec = 0;
    uint32_t myval = 0;
    uint32_t blocker = 0;   // the earlier seed whose claim stopped the grow
    bool done = false, conflict = false;
  };

  uint8_t dummy = 0;

  bool start(Grow& g, int sx, int sy, double prec_, uint32_t myval) {
    g = Grow();
    g.prec = prec_;
    g.myval = myval;
    uint32_t& s = stamp[(size_t)sy * W + sx];
    if (s == 0 || (s >> 1) < (myval >> 1)) {   // USED or an earlier seed's claim
      g.conflict = g.done = true;
      g.blocker = s >> 1;
      return false;
    }
    s = std::min(s, myval);
    RegionPoint rp{sx, sy, &dummy, L.ang(sx, sy), L.modgrad[(size_t)sy * W + sx]};
    g.reg.push_back(rp);
    g.reg_angle = rp.angle;
    g.sumdx = float(pmath::cos_(g.reg_angle));
    g.sumdy = float(pmath::sin_(g.reg_angle));
    return true;
  }

  // one point expansion with the neighbour stamps read at the step's start
  void step(Grow& g, const uint32_t* snap) {
    if (g.done) return;
    if (g.i >= g.reg.size()) {
      g.done = true;
      return;
    }
    const RegionPoint rpoint = g.reg[g.i];
    const int xx_min = std::max(rpoint.x - 1, 0), xx_max = std::min(rpoint.x + 1, W - 1);
    const int yy_min = std::max(rpoint.y - 1, 0), yy_max = std::min(rpoint.y + 1, H - 1);
    for (int yy = yy_min; yy <= yy_max; ++yy)
      for (int xx = xx_min; xx <= xx_max; ++xx) {
        if (xx == rpoint.x && yy == rpoint.y) continue;
        const int k = (yy - rpoint.y + 1) * 3 + (xx - rpoint.x + 1);
        const uint32_t s = snap[k];
        if (s == 0 || s == g.myval) continue;
        if (!L.isAligned(xx, yy, g.reg_angle, g.prec)) continue;
        if ((s >> 1) < (g.myval >> 1)) {
          g.conflict = g.done = true;
          g.blocker = s >> 1;
          return;
        }
        uint32_t& st = stamp[(size_t)yy * W + xx];
        st = std::min(st, g.myval);
        const double angle = L.ang(xx, yy);
        g.reg.push_back(RegionPoint{xx, yy, &dummy, angle, L.modgrad[(size_t)yy * W + xx]});
        g.sumdx += cosf_cr(float(angle));
        g.sumdy += sinf_cr(float(angle));
        g.reg_angle = oracle_fast_atan2(g.sumdy, g.sumdx) * DEG_TO_RADS;
      }
    g.i++;
    if (g.i >= g.reg.size()) g.done = true;
  }

  void snapshot(const Grow& g, uint32_t* snap) const {
    if (g.done || g.i >= g.reg.size()) return;
    const RegionPoint& r = g.reg[g.i];
    for (int k = 0; k < 9; k++) {
      const int xx = r.x + k % 3 - 1, yy = r.y + k / 3 - 1;
      snap[k] = (xx >= 0 && yy >= 0 && xx < W && yy < H) ? stamp[(size_t)yy * W + xx] : 0;
    }
  }
};

enum { kFresh, kGrow1, kWaitRect1, kGrow2, kWaitRect2, kDone, kConflict };
enum { kSmall, kFail, kCand, kSkip };

struct Slot {
  int pos = 0, x = 0, y = 0;
  uint32_t tag = 0;
  int state = kFresh;
  int lane = -1;
  int result = kSmall;
  Sim::Grow g1, g2;
  std::vector<int> touched;       // pixel indices ever claimed
  std::vector<RegionPoint> fin;   // the final region
  Rect rec{};
  bool requeue = false;
  uint32_t blocker = 0;   // kConflict: re-fetch once every seed up to it is committed
};

struct Stats {
  long long iters = 0, grow_iters = 0, fits = 0, fit_batches = 0, commits = 0, regrows = 0,
            conflicts = 0, fetched = 0, skipped_at_head = 0, stalls = 0;
  double cycles = 0, cyc_grow = 0, cyc_fit = 0, cyc_commit = 0;
  long long head_state[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // per iteration with stalls: the head's state
};

// the fit's first pass phase (region2rect of the first region, refine's
// density test and angle statistics, lsd.cpp): true = a second grow is
// needed (started here with tau); otherwise the result is final. passes =
// wave-wide passes over the list this phase costs.
static bool rect1(Sim& S, Slot& s, int& passes) {
  LSD& L = S.L;
  std::vector<RegionPoint>& reg = s.g1.reg;
  Rect rec;
  L.region2rect(reg, s.g1.reg_angle, S.prec, S.p, rec);
  passes = 3;
  double density = double(reg.size()) / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
  if (density >= L.DENSITY_TH) {
    s.rec = rec;
    s.result = kCand;
    s.fin = reg;
    return false;
  }
  passes++;
  const double xc = double(reg[0].x), yc = double(reg[0].y);
  const double ang_c = reg[0].angle;
  double sum = 0, s_sum = 0;
  int n = 0;
  for (size_t i = 0; i < reg.size(); ++i)
    if (dist(xc, yc, reg[i].x, reg[i].y) < rec.width) {
      const double ang_d = angle_diff_signed(reg[i].angle, ang_c);
      sum += ang_d;
      s_sum += ang_d * ang_d;
      ++n;
    }
  const double mean_angle = sum / double(n);
  const double tau = 2.0 * std::sqrt((s_sum - 2.0 * mean_angle * sum) / double(n) + mean_angle * mean_angle);
  S.start(s.g2, reg[0].x, reg[0].y, tau, s.tag << 1);
  return true;
}

// the fit's second pass phase: region2rect of the second region and
// reduce_region_radius
static void rect2(Sim& S, Slot& s, int& passes) {
  LSD& L = S.L;
  std::vector<RegionPoint> r2 = s.g2.reg;
  double reg_angle = s.g2.reg_angle;
  passes = 0;
  if (r2.size() < 2) {
    s.result = kFail;
    s.fin = r2;
    return;
  }
  Rect rec;
  L.region2rect(r2, reg_angle, S.prec, S.p, rec);
  passes = 3;
  const double density = double(r2.size()) / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
  bool ok = true;
  if (density < L.DENSITY_TH) {
    const size_t n0 = r2.size();
    ok = L.reduce_region_radius(r2, reg_angle, S.prec, S.p, rec, density);
    passes += 6 + int(2 * (n0 - r2.size()) / std::max<size_t>(1, n0 / 8));   // rough: a few iterations
  }
  s.fin = r2;
  s.result = ok ? kCand : kFail;
  s.rec = rec;
}

struct Result {
  std::vector<Rect> cands;
  Stats st;
};

// the streaming schedule
static Result run_stream(LSD& L, double prec, double p, size_t min_reg, int window, int fit_batch,
                         const Cost& C) {
  Sim S(L, prec, p, min_reg);
  Result R;
  Stats& st = R.st;
  const int nl = (int)L.ordered.size();
  std::deque<Slot> win;        // [head, ...]: fetched, uncommitted seeds in fetch order
  long long head_tag = 0;      // tag of win.front()
  int scan = 0;
  uint32_t next_tag = 1;       // 0 is USED
  std::vector<Slot*> lane(64, nullptr);
  std::vector<uint32_t> snapbuf;
  auto is_used = [&](int x, int y) { return S.stamp[(size_t)y * S.W + x] == 0; };
  while (true) {
    st.iters++;
    // 1. idle lanes take work: the head's regrow first, then new seeds
    for (int l = 0; l < 64; l++) {
      if (lane[l]) continue;
      // a conflicted seed whose blocker has committed is taken first (in
      // window order): skipped at once if its seed pixel is now USED, else
      // regrown (speculatively, exact once it is the head)
      Slot* pick = nullptr;
      const uint32_t htag = win.empty() ? next_tag : win.front().tag;
      for (Slot& sl : win) {
        if (sl.state == kConflict && sl.lane < 0 && sl.blocker < htag) {
          if (is_used(sl.x, sl.y)) {
            sl.state = kDone;
            sl.result = kSkip;
            sl.touched.clear();
            sl.fin.clear();
            continue;
          }
          pick = &sl;
          st.regrows++;
          break;
        }
      }
      if (!pick) {
        if ((int)win.size() >= window) {
          st.stalls++;
          continue;
        }
        while (scan < nl) {
          const int x = L.ordered[scan].x, y = L.ordered[scan].y;
          const int i = scan++;
          if (i % 64 == 0) st.cycles += C.scan64 / 64.0 * 0;   // scans are batched below
          if (is_used(x, y) || L.ang(x, y) == NOTDEF) continue;
          win.emplace_back();
          Slot& s = win.back();
          s.pos = i;
          s.x = x;
          s.y = y;
          s.tag = next_tag++;
          pick = &s;
          st.fetched++;
          break;
        }
        if (!pick) continue;
      }
      pick->lane = l;
      pick->requeue = false;
      pick->blocker = 0;
      pick->state = kGrow1;
      pick->touched.clear();
      pick->fin.clear();
      S.start(pick->g1, pick->x, pick->y, prec, (pick->tag << 1) | 1u);
      if (!pick->g1.conflict) pick->touched.push_back(pick->y * S.W + pick->x);
      lane[l] = pick;
    }
    // 2. one lockstep grow step for every growing lane (first or refine's
    // second grow; stamps read first)
    bool grew = false;
    uint32_t snaps[64][9];
    auto growing = [](const Slot* s) { return s && (s->state == kGrow1 || s->state == kGrow2); };
    for (int l = 0; l < 64; l++)
      if (growing(lane[l])) S.snapshot(lane[l]->state == kGrow1 ? lane[l]->g1 : lane[l]->g2, snaps[l]);
    auto abort_slot = [&](Slot* s, int l, uint32_t blocker) {
      s->state = kConflict;
      s->blocker = blocker;
      for (int px : s->touched)
        if (S.stamp[px] != 0 && (S.stamp[px] >> 1) == s->tag) S.stamp[px] = kFree;
      s->touched.clear();
      s->lane = -1;
      lane[l] = nullptr;
      st.conflicts++;
    };
    for (int l = 0; l < 64; l++) {
      Slot* s = lane[l];
      if (!growing(s)) continue;
      grew = true;
      Sim::Grow& g = s->state == kGrow1 ? s->g1 : s->g2;
      const size_t before = g.reg.size();
      S.step(g, snaps[l]);
      for (size_t k = before; k < g.reg.size(); k++)
        s->touched.push_back(g.reg[k].y * S.W + g.reg[k].x);
      if (!g.done) continue;
      if (g.conflict) {
        abort_slot(s, l, g.blocker);
      } else if (s->state == kGrow1 && g.reg.size() < min_reg) {
        s->result = kSmall;
        s->fin = g.reg;
        s->state = kDone;
        s->lane = -1;
        lane[l] = nullptr;
      } else {
        s->state = s->state == kGrow1 ? kWaitRect1 : kWaitRect2;
      }
    }
    if (grew) {
      st.grow_iters++;
      st.cycles += C.step;
      st.cyc_grow += C.step;
    }
    // 3. a pass batch: the waiting fit phases, wave-wide passes in groups of 4
    int nwait = 0;
    bool any_grow = false;
    for (int l = 0; l < 64; l++)
      if (lane[l]) {
        nwait += lane[l]->state == kWaitRect1 || lane[l]->state == kWaitRect2;
        any_grow |= growing(lane[l]);
      }
    const bool head_waits = !win.empty() && (win.front().state == kWaitRect1 ||
                                             win.front().state == kWaitRect2);
    if (nwait > 0 && (nwait >= fit_batch || head_waits || !any_grow)) {
      st.fit_batches++;
      double cyc = C.fit_fixed;
      std::vector<std::pair<int, size_t>> work;   // (passes, list length)
      for (int l = 0; l < 64; l++) {
        Slot* s = lane[l];
        if (!s || (s->state != kWaitRect1 && s->state != kWaitRect2)) continue;
        int passes = 0;
        if (s->state == kWaitRect1) {
          st.fits++;
          const bool again = rect1(S, *s, passes);
          work.emplace_back(passes, s->g1.reg.size());
          if (!again) {
            s->state = kDone;
            s->lane = -1;
            lane[l] = nullptr;
          } else if (s->g2.conflict) {
            abort_slot(s, l, s->g2.blocker);
          } else {
            s->touched.push_back(s->g2.reg[0].y * S.W + s->g2.reg[0].x);
            s->state = kGrow2;
          }
        } else {
          rect2(S, *s, passes);
          work.emplace_back(passes, s->g2.reg.size());
          s->state = kDone;
          s->lane = -1;
          lane[l] = nullptr;
        }
      }
      std::sort(work.begin(), work.end(), [](auto& a, auto& b) { return a.second < b.second; });
      for (size_t g = 0; g < work.size(); g += 4) {
        int mp = 0;
        size_t mx = 0;
        for (size_t k = g; k < std::min(work.size(), g + 4); k++) {
          mp = std::max(mp, work[k].first);
          mx = std::max(mx, work[k].second);
        }
        cyc += mp * C.pass64 * double((mx + 63) / 64);
      }
      st.cycles += cyc;
      st.cyc_fit += cyc;
    }
    // 4. commit from the head
    while (!win.empty()) {
      Slot& h = win.front();
      if (h.state == kDone && h.result == kSkip) {
        st.skipped_at_head++;
        st.cycles += C.commit_seed;
        st.cyc_commit += C.commit_seed;
        win.pop_front();
        continue;
      }
      if (h.state != kDone) break;
      // re-check: every touched pixel still carries the own tag
      bool ok = true;
      for (int px : h.touched)
        if ((S.stamp[px] >> 1) != h.tag || S.stamp[px] == 0) ok = false;
      st.cycles += C.commit_seed + C.commit_px * double(h.touched.size());
      st.cyc_commit += C.commit_seed + C.commit_px * double(h.touched.size());
      if (!ok) {
        for (int px : h.touched)
          if (S.stamp[px] != 0 && (S.stamp[px] >> 1) == h.tag) S.stamp[px] = kFree;
        h.touched.clear();
        h.state = kConflict;
        h.blocker = 0;   // every earlier seed is committed: eligible now
        h.lane = -1;
        st.conflicts++;
        break;
      }
      for (const RegionPoint& r : h.fin) S.stamp[(size_t)r.y * S.W + r.x] = 0;
      for (int px : h.touched)
        if (S.stamp[px] != 0 && (S.stamp[px] >> 1) == h.tag) S.stamp[px] = kFree;
      if (h.result == kCand) R.cands.push_back(h.rec);
      st.commits++;
      win.pop_front();
    }
    bool busy = false;
    int idle = 0;
    for (int l = 0; l < 64; l++) {
      busy |= lane[l] != nullptr;
      idle += lane[l] == nullptr;
    }
    if (idle > 32 && !win.empty()) st.head_state[win.front().state]++;
    if (!busy && win.empty() && scan >= nl) break;
    if (st.iters > 2000000) {
      fprintf(stderr, "no progress\n");
      break;
    }
  }
  st.cycles += C.scan64 * double(nl) / 64.0;
  return R;
}

// the sequential loop's candidates (lsd.cpp flsd, rectangles after refine)
static std::vector<Rect> sequential(LSD& L, double prec, double p, size_t min_reg,
                                    std::vector<std::vector<int>>* regions) {
  std::vector<Rect> out;
  L.used.assign((size_t)L.img_width * L.img_height, NOTUSED);
  std::vector<RegionPoint> reg;
  for (size_t i = 0; i < L.ordered.size(); ++i) {
    const int px = L.ordered[i].x, py = L.ordered[i].y;
    if (L.used[(size_t)py * L.img_width + px] != NOTUSED || L.ang(px, py) == NOTDEF) continue;
    double reg_angle;
    L.region_grow(px, py, reg, reg_angle, prec);
    if (regions) {
      regions->emplace_back();
      for (auto& r : reg) regions->back().push_back(r.y * L.img_width + r.x);
    }
    if (reg.size() < min_reg) continue;
    Rect rec;
    L.region2rect(reg, reg_angle, prec, p, rec);
    if (!L.refine(reg, reg_angle, prec, p, rec)) continue;
    out.push_back(rec);
  }
  return out;
}

}  // namespace lsdo

extern "C" int lsd_stream_sim(const uint8_t* img, int W, int H, int window, int fit_batch,
                              double* out16, double* out4) {
  using namespace lsdo;
  LSD L;
  const double prec = kPi * L.ANG_TH / 180;
  const double p = L.ANG_TH / 180;
  const double rho = L.QUANT / pmath::sin_(prec);
  const double sigma = (L.SCALE < 1) ? (L.SIGMA_SCALE / L.SCALE) : L.SIGMA_SCALE;
  const unsigned h = (unsigned)std::ceil(sigma * std::sqrt(2 * 3.0 * pmath::log_(10.0)));
  const int ksize = 1 + 2 * (int)h;
  std::vector<int> k(ksize);
  fixed_gauss_kernel(ksize, sigma, k.data());
  std::vector<uint8_t> g((size_t)W * H);
  gauss_fixed(img, W, H, k.data(), ksize, g.data());
  L.img_width = (int)std::lrint(W * L.SCALE);
  L.img_height = (int)std::lrint(H * L.SCALE);
  L.scaled.assign((size_t)L.img_width * L.img_height, 0);
  resize_exact(g.data(), W, H, L.SCALE, L.scaled.data(), L.img_width, L.img_height);
  L.ll_angle(rho);
  L.LOG_NT = 5 * (pmath::log10_(double(L.img_width)) + pmath::log10_(double(L.img_height))) / 2 +
             pmath::log10_(11.0);
  const size_t min_reg = size_t(-L.LOG_NT / pmath::log10_(p));
  // the sequential reference, and its round-synchronous cost model: rounds of
  // 64 consecutive grown seeds, each costing its slowest grow + its fits
  std::vector<std::vector<int>> regions;
  const std::vector<Rect> ref = sequential(L, prec, p, min_reg, &regions);
  {
    std::vector<size_t> sz;
    for (auto& r : regions) sz.push_back(r.size());
    std::sort(sz.rbegin(), sz.rend());
    size_t big = 0, nbig = 0, tot = 0;
    for (size_t v : sz) {
      tot += v;
      if (v >= 100) { big += v; nbig++; }
    }
    fprintf(stderr, "regions %zu, points %zu, >=100: %zu regions %zu points; top:", sz.size(), tot, nbig, big);
    for (size_t i = 0; i < std::min<size_t>(12, sz.size()); i++) fprintf(stderr, " %zu", sz[i]);
    fprintf(stderr, "\n");
  }
  Cost C;
  double round_cycles = 0;
  for (size_t r0 = 0; r0 < regions.size(); r0 += 64) {
    size_t mx = 0;
    int nfit = 0;
    size_t fitn = 0;
    for (size_t i = r0; i < std::min(regions.size(), r0 + 64); i++) {
      mx = std::max(mx, regions[i].size());
      if (regions[i].size() >= min_reg) {
        nfit++;
        fitn = std::max(fitn, regions[i].size());
      }
    }
    round_cycles += C.step * double(mx) + C.commit_seed * 64;
    if (nfit) round_cycles += C.fit_fixed + 8 * C.pass64 * double((nfit + 3) / 4) * double((fitn + 63) / 64) +
                              C.step * double(fitn);
  }
  round_cycles += C.scan64 * double(L.ordered.size()) / 64.0;
  Result R = run_stream(L, prec, p, min_reg, window, fit_batch, C);
  bool same = R.cands.size() == ref.size();
  for (size_t i = 0; same && i < ref.size(); i++)
    same = std::memcmp(&R.cands[i], &ref[i], sizeof(Rect)) == 0;
  const Stats& s = R.st;
  const double v[16] = {double(same), double(ref.size()), double(R.cands.size()), double(regions.size()),
                        double(s.iters), double(s.grow_iters), double(s.fits), double(s.fit_batches),
                        double(s.commits), double(s.regrows), double(s.conflicts), double(s.fetched),
                        double(s.skipped_at_head), s.cycles, round_cycles, double(s.stalls)};
  std::memcpy(out16, v, sizeof(v));
  out4[0] = s.cyc_grow;
  out4[1] = s.cyc_fit;
  out4[2] = s.cyc_commit;
  out4[3] = 0;
  fprintf(stderr, "head states at iterations with > 32 idle lanes: grow1 %lld rect1 %lld grow2 %lld rect2 %lld done %lld conflict %lld\n",
          s.head_state[kGrow1], s.head_state[kWaitRect1], s.head_state[kGrow2], s.head_state[kWaitRect2],
          s.head_state[kDone], s.head_state[kConflict]);
  return 0;
}
