// Tracking::Tracking's settings read (Tracking.cc:53-147) from an OpenCV
// FileStorage YAML file (Examples/RGB-D/TUM1.yaml:8-55), host C++: the flat
// "Key.name: value" subset the reference's settings files use, read with
// OpenCV 3.4's FileNode conversions (readInt / readReal: a missing key reads
// 0, a real read as int is cvRound-ed, a string reads 0x7fffffff / 1e300).
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>

#include "../../include/orbpl.h"
#include <hip/hip_runtime.h>

#include "orbpl_runtime.h"

namespace {

struct Node {
  enum Kind { kInt, kReal, kString } kind = kString;
  long long i = 0;
  double f = 0;
};

std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t' || s[a] == '\r')) a++;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r')) b--;
  return s.substr(a, b - a);
}

Node parse_value(const std::string& v) {
  Node n;
  if (v.empty()) return n;
  if (v[0] == '"' || v[0] == '\'') return n;   // a string
  char* end = nullptr;
  errno = 0;
  const long long iv = strtoll(v.c_str(), &end, 10);
  if (end && *end == '\0' && errno == 0) {
    n.kind = Node::kInt;
    n.i = iv;
    n.f = (double)iv;
    return n;
  }
  end = nullptr;
  const double fv = strtod(v.c_str(), &end);
  if (end && *end == '\0') {
    n.kind = Node::kReal;
    n.f = fv;
  }
  return n;
}

struct Settings {
  std::map<std::string, Node> kv;
  // cv::FileNode::operator int / float of OpenCV 3.4 (readInt / readReal)
  int geti(const char* k) const {
    auto it = kv.find(k);
    if (it == kv.end()) return 0;
    const Node& n = it->second;
    if (n.kind == Node::kInt) return (int)n.i;
    if (n.kind == Node::kReal) return (int)std::nearbyint(n.f);   // cvRound
    return 0x7fffffff;
  }
  float getf(const char* k) const {
    auto it = kv.find(k);
    if (it == kv.end()) return 0.0f;
    const Node& n = it->second;
    if (n.kind == Node::kString) return (float)1e300;
    return (float)n.f;
  }
};

bool read_settings(const char* path, Settings* s) {
  FILE* fp = fopen(path, "rb");
  if (!fp) return false;
  std::string line;
  int c;
  auto flush = [&]() {
    // drop a comment (outside quotes), the %YAML header and document markers
    std::string t;
    bool q = false;
    for (char ch : line) {
      if (ch == '"' || ch == '\'') q = !q;
      if (ch == '#' && !q) break;
      t.push_back(ch);
    }
    t = trim(t);
    line.clear();
    if (t.empty() || t[0] == '%' || t == "---" || t == "...") return;
    const size_t colon = t.find(':');
    if (colon == std::string::npos) return;
    const std::string k = trim(t.substr(0, colon)), v = trim(t.substr(colon + 1));
    if (!k.empty()) s->kv[k] = parse_value(v);
  };
  while ((c = fgetc(fp)) != EOF) {
    if (c == '\n') flush();
    else line.push_back((char)c);
  }
  flush();
  fclose(fp);
  return true;
}

}  // namespace

extern "C" {

int orbpl_settings_load(const char* path, int sensor, orbpl_settings* out) {
  if (!path || !out) return orbpl::arg_fail("orbpl_settings_load: NULL argument");
  if (sensor < ORBPL_SENSOR_MONOCULAR || sensor > ORBPL_SENSOR_RGBD)
    return orbpl::arg_fail("orbpl_settings_load: sensor out of range");
  Settings s;
  if (!read_settings(path, &s)) return orbpl::arg_fail("orbpl_settings_load: cannot open the file");
  orbpl_settings r;
  std::memset(&r, 0, sizeof(r));
  // Tracking.cc:56-75: K, DistCoef (k3 kept only when non-zero; 0 either way here)
  r.cam.fx = s.getf("Camera.fx");
  r.cam.fy = s.getf("Camera.fy");
  r.cam.cx = s.getf("Camera.cx");
  r.cam.cy = s.getf("Camera.cy");
  r.cam.k1 = s.getf("Camera.k1");
  r.cam.k2 = s.getf("Camera.k2");
  r.cam.p1 = s.getf("Camera.p1");
  r.cam.p2 = s.getf("Camera.p2");
  r.cam.k3 = s.getf("Camera.k3");
  r.cam.bf = s.getf("Camera.bf");   // mbf (Tracking.cc:79)
  // the image size is the images' in the reference; the files carry it
  r.cam.width = s.geti("Camera.width");
  r.cam.height = s.geti("Camera.height");
  // Tracking.cc:81-87: fps 0 -> 30, mMaxFrames = fps
  float fps = s.getf("Camera.fps");
  if (fps == 0) fps = 30;
  r.fps = fps;
  r.max_frames = (int)fps;
  r.rgb = s.geti("Camera.RGB");
  // Tracking.cc:113-117
  r.orb.nfeatures = s.geti("ORBextractor.nFeatures");
  r.orb.scale_factor = s.getf("ORBextractor.scaleFactor");
  r.orb.nlevels = s.geti("ORBextractor.nLevels");
  r.orb.ini_th_fast = s.geti("ORBextractor.iniThFAST");
  r.orb.min_th_fast = s.geti("ORBextractor.minThFAST");
  // Tracking.cc:134-138: mThDepth = mbf * ThDepth / fx (stereo / RGB-D)
  if (sensor != ORBPL_SENSOR_MONOCULAR)
    r.cam.th_depth = r.cam.bf * s.getf("ThDepth") / r.cam.fx;
  // Tracking.cc:140-146: mDepthMapFactor (RGB-D)
  r.depth_map_factor = 1.0f;
  if (sensor == ORBPL_SENSOR_RGBD) {
    const float f = s.getf("DepthMapFactor");
    r.depth_map_factor_setting = f;
    r.depth_map_factor = std::fabs(f) < 1e-5 ? 1.0f : 1.0f / f;
  }
  *out = r;
  return ORBPL_OK;
}

}  // extern "C"
