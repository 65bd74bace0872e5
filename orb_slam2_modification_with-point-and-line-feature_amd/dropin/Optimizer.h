// Drop-in ORB_SLAM2::Optimizer pose-only entry points (include/Optimizer.h:121,
// 234; src/Optimizer.cc:375-619, 2132-2486) over orbpl_pose_optimization.
#pragma once
#include "Frame.h"

namespace ORB_SLAM2 {

class Optimizer {
 public:
  int static PoseOptimization(Frame* pFrame);
  int static PoseOptimizationWithLines(Frame* pFrame);
};

}  // namespace ORB_SLAM2
