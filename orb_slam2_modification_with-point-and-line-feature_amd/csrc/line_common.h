// Device helpers shared by the line kernels (KeyLine fields recomputed from
// end points: LSDDetector::detectImpl, Frame::UndistortKeyLines,
// LineMatcher::UpdateKeyLineData).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/orbpl.h"
#include "lsd_math.h"

namespace orbpl {

// cv::LineIterator(img(W x H), Point(cvRound), Point(cvRound), 8).count
__device__ inline int line_iterator_count(int W, int H, float fx1, float fy1, float fx2, float fy2) {
  long long x1 = (long long)rintf(fx1), y1 = (long long)rintf(fy1);
  long long x2 = (long long)rintf(fx2), y2 = (long long)rintf(fy2);
  if ((unsigned long long)x1 >= (unsigned long long)W || (unsigned long long)x2 >= (unsigned long long)W ||
      (unsigned long long)y1 >= (unsigned long long)H || (unsigned long long)y2 >= (unsigned long long)H) {
    // clipLine (drawing.cpp)
    const long long right = W - 1, bottom = H - 1;
    int c1 = (x1 < 0) + (x1 > right) * 2 + (y1 < 0) * 4 + (y1 > bottom) * 8;
    int c2 = (x2 < 0) + (x2 > right) * 2 + (y2 < 0) * 4 + (y2 > bottom) * 8;
    if ((c1 & c2) == 0 && (c1 | c2) != 0) {
      long long a;
      if (c1 & 12) {
        a = c1 < 8 ? 0 : bottom;
        x1 += (long long)((double)(a - y1) * (x2 - x1) / (y2 - y1));
        y1 = a;
        c1 = (x1 < 0) + (x1 > right) * 2;
      }
      if (c2 & 12) {
        a = c2 < 8 ? 0 : bottom;
        x2 += (long long)((double)(a - y2) * (x2 - x1) / (y2 - y1));
        y2 = a;
        c2 = (x2 < 0) + (x2 > right) * 2;
      }
      if ((c1 & c2) == 0 && (c1 | c2) != 0) {
        if (c1) {
          a = c1 == 1 ? 0 : right;
          y1 += (long long)((double)(a - x1) * (y2 - y1) / (x2 - x1));
          x1 = a;
          c1 = 0;
        }
        if (c2) {
          a = c2 == 1 ? 0 : right;
          y2 += (long long)((double)(a - x2) * (y2 - y1) / (x2 - x1));
          x2 = a;
          c2 = 0;
        }
      }
    }
    if ((c1 | c2) != 0) return 0;
  }
  long long dx = x2 - x1, dy = y2 - y1;
  if (dx < 0) dx = -dx;
  if (dy < 0) dy = -dy;
  return (int)(dx > dy ? dx : dy) + 1;
}

// lineLength, numOfPixels (LineIterator on the W x H image), angle (atan2f,
// pinned P12), size, response, pt from the end points.
__device__ inline void refresh_keyline(orbpl_keyline& kl, int W, int H) {
  kl.pt_x = (kl.endPointX + kl.startPointX) / 2;
  kl.pt_y = (kl.endPointY + kl.startPointY) / 2;
  const double dx = (double)(kl.startPointX - kl.endPointX), dy = (double)(kl.startPointY - kl.endPointY);
  kl.lineLength = float(sqrt(dx * dx + dy * dy));
  kl.numOfPixels = line_iterator_count(W, H, kl.startPointX, kl.startPointY, kl.endPointX, kl.endPointY);
  kl.angle = (float)lsdm::atan2_((double)(kl.endPointY - kl.startPointY),
                                 (double)(kl.endPointX - kl.startPointX));
  kl.size = (kl.endPointX - kl.startPointX) * (kl.endPointY - kl.startPointY);
  kl.response = kl.lineLength / (float)max(W, H);
}

}  // namespace orbpl
