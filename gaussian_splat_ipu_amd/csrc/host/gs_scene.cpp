// gs_scene.cpp -- host-side data path: PLY/XYZ ingest, synthetic scenes and
// the render server's scene preparation.
//
//   loadPoints / loadPlyFile / loadXyz / fillPlyProperties   src/splat/file_io.cpp:11-77
//   scene preparation (centre, negate z, SH DC colour)        src/main/splat.cpp:83-163
//   synthetic generator (seeded, INRIA layout)                SURVEY.md §8 d
//
// The reference parses PLY with the vendored happly.h; this is an independent
// binary/ascii PLY reader that keeps every vertex property as float (so the
// f_rest_* SH coefficients pass through) and enforces the same required set
// as fillPlyProperties.
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstring>
#include <fstream>
#include <limits>
#include <memory>
#include <mutex>
#include <sstream>

#include "gs_host.hpp"

namespace gsh {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
const char* last_error() { return g_last_error.c_str(); }

namespace {

enum class PType { I8, U8, I16, U16, I32, U32, F32, F64, BAD };

PType parse_type(const std::string& t) {
  if (t == "char" || t == "int8") return PType::I8;
  if (t == "uchar" || t == "uint8") return PType::U8;
  if (t == "short" || t == "int16") return PType::I16;
  if (t == "ushort" || t == "uint16") return PType::U16;
  if (t == "int" || t == "int32") return PType::I32;
  if (t == "uint" || t == "uint32") return PType::U32;
  if (t == "float" || t == "float32") return PType::F32;
  if (t == "double" || t == "float64") return PType::F64;
  return PType::BAD;
}

size_t type_size(PType t) {
  switch (t) {
    case PType::I8: case PType::U8: return 1;
    case PType::I16: case PType::U16: return 2;
    case PType::I32: case PType::U32: case PType::F32: return 4;
    case PType::F64: return 8;
    default: return 0;
  }
}

struct Prop {
  std::string name;
  PType type = PType::BAD;
  bool is_list = false;
  PType count_type = PType::BAD;
};

struct Element {
  std::string name;
  int64_t count = 0;
  std::vector<Prop> props;
};

template <typename T>
T load_le(const unsigned char* p, bool big) {
  unsigned char b[sizeof(T)];
  if (big) {
    for (size_t i = 0; i < sizeof(T); ++i) b[i] = p[sizeof(T) - 1 - i];
  } else {
    std::memcpy(b, p, sizeof(T));
  }
  T v;
  std::memcpy(&v, b, sizeof(T));
  return v;
}

double read_bin(const unsigned char* p, PType t, bool big) {
  switch (t) {
    case PType::I8: return (double)(int8_t)p[0];
    case PType::U8: return (double)p[0];
    case PType::I16: return (double)load_le<int16_t>(p, big);
    case PType::U16: return (double)load_le<uint16_t>(p, big);
    case PType::I32: return (double)load_le<int32_t>(p, big);
    case PType::U32: return (double)load_le<uint32_t>(p, big);
    case PType::F32: return (double)load_le<float>(p, big);
    case PType::F64: return load_le<double>(p, big);
    default: return 0.0;
  }
}

float to_float(double v, PType t) {
  // float properties are copied bit-for-bit; others converted
  return (float)v;
  (void)t;
}

bool ends_with_ci(const std::string& s, const std::string& ext) {
  if (s.size() < ext.size()) return false;
  for (size_t i = 0; i < ext.size(); ++i)
    if (std::tolower((unsigned char)s[s.size() - ext.size() + i]) != ext[i]) return false;
  return true;
}

int load_ply(const std::string& path, gs_ply& out) {
  std::ifstream in(path, std::ios::binary);
  if (!in) {
    set_error("cannot open " + path);
    return GS_EIO;
  }
  std::string line;
  std::getline(in, line);
  if (line.rfind("ply", 0) != 0) {
    set_error(path + ": not a PLY file");
    return GS_EIO;
  }
  std::string format;
  std::vector<Element> elems;
  while (std::getline(in, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    std::istringstream ss(line);
    std::string tok;
    ss >> tok;
    if (tok == "format") {
      ss >> format;
    } else if (tok == "element") {
      Element e;
      ss >> e.name >> e.count;
      elems.push_back(e);
    } else if (tok == "property") {
      if (elems.empty()) {
        set_error(path + ": property before element");
        return GS_EIO;
      }
      Prop p;
      std::string t;
      ss >> t;
      if (t == "list") {
        std::string ct, vt;
        ss >> ct >> vt >> p.name;
        p.is_list = true;
        p.count_type = parse_type(ct);
        p.type = parse_type(vt);
      } else {
        p.type = parse_type(t);
        ss >> p.name;
      }
      if (p.type == PType::BAD || (p.is_list && p.count_type == PType::BAD)) {
        set_error(path + ": unsupported property type in '" + line + "'");
        return GS_EIO;
      }
      elems.back().props.push_back(p);
    } else if (tok == "end_header") {
      break;
    }
  }
  const bool ascii = format == "ascii";
  const bool big = format == "binary_big_endian";
  if (!ascii && !big && format != "binary_little_endian") {
    set_error(path + ": unsupported PLY format '" + format + "'");
    return GS_EIO;
  }
  bool found = false;
  for (const Element& e : elems) {
    const bool is_vertex = e.name == "vertex";
    if (is_vertex) {
      out.n = e.count;
      for (const Prop& p : e.props)
        if (!p.is_list) out.add(p.name);
      found = true;
    }
    std::vector<std::vector<float>*> cols;
    for (const Prop& p : e.props) cols.push_back((is_vertex && !p.is_list) ? &out.props[p.name] : nullptr);
    if (ascii) {
      for (int64_t i = 0; i < e.count; ++i) {
        for (size_t k = 0; k < e.props.size(); ++k) {
          const Prop& p = e.props[k];
          if (p.is_list) {
            double cnt;
            in >> cnt;
            for (int64_t j = 0; j < (int64_t)cnt; ++j) {
              double v;
              in >> v;
            }
          } else {
            double v;
            in >> v;
            if (cols[k]) (*cols[k])[(size_t)i] = to_float(v, p.type);
          }
        }
        if (!in) {
          set_error(path + ": truncated ascii data");
          return GS_EIO;
        }
      }
    } else {
      // fast path: fixed-size records
      bool fixed = true;
      size_t rec = 0;
      for (const Prop& p : e.props) {
        if (p.is_list) fixed = false;
        rec += type_size(p.type);
      }
      if (fixed) {
        std::vector<unsigned char> buf(rec * (size_t)std::min<int64_t>(e.count, 1 << 16));
        int64_t done = 0;
        while (done < e.count) {
          const int64_t chunk = std::min<int64_t>(e.count - done, 1 << 16);
          in.read((char*)buf.data(), (std::streamsize)(rec * chunk));
          if (!in) {
            set_error(path + ": truncated binary data");
            return GS_EIO;
          }
          for (int64_t i = 0; i < chunk; ++i) {
            const unsigned char* r = buf.data() + rec * i;
            size_t off = 0;
            for (size_t k = 0; k < e.props.size(); ++k) {
              const Prop& p = e.props[k];
              if (cols[k]) {
                if (p.type == PType::F32 && !big) {
                  float f;
                  std::memcpy(&f, r + off, 4);
                  (*cols[k])[(size_t)(done + i)] = f;
                } else {
                  (*cols[k])[(size_t)(done + i)] = to_float(read_bin(r + off, p.type, big), p.type);
                }
              }
              off += type_size(p.type);
            }
          }
          done += chunk;
        }
      } else {
        for (int64_t i = 0; i < e.count; ++i) {
          for (size_t k = 0; k < e.props.size(); ++k) {
            const Prop& p = e.props[k];
            unsigned char b[8];
            if (p.is_list) {
              in.read((char*)b, (std::streamsize)type_size(p.count_type));
              const int64_t cnt = (int64_t)read_bin(b, p.count_type, big);
              in.seekg((std::streamoff)(cnt * (int64_t)type_size(p.type)), std::ios::cur);
            } else {
              in.read((char*)b, (std::streamsize)type_size(p.type));
              if (cols[k]) (*cols[k])[(size_t)i] = to_float(read_bin(b, p.type, big), p.type);
            }
          }
          if (!in) {
            set_error(path + ": truncated binary data");
            return GS_EIO;
          }
        }
      }
    }
    if (is_vertex) break;  // nothing after the vertex element is needed
  }
  if (!found) {
    set_error(path + ": no vertex element");
    return GS_EIO;
  }
  // fillPlyProperties (file_io.cpp:62-77) requires all 14 properties
  static const char* required[] = {"x", "y", "z", "f_dc_0", "f_dc_1", "f_dc_2", "opacity",
                                   "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2",
                                   "rot_3"};
  for (const char* r : required) {
    if (!out.get(r)) {
      set_error(path + ": missing required vertex property '" + r + "'");
      return GS_EIO;
    }
  }
  return GS_OK;
}

int load_xyz(const std::string& path, gs_ply& out) {
  // splat::loadXyz (file_io.cpp:11-28): one "x y z" point per line
  std::ifstream in(path);
  if (!in) {
    set_error("cannot open " + path);
    return GS_EIO;
  }
  std::vector<float> x, y, z;
  for (std::string line; std::getline(in, line);) {
    std::stringstream ss(line);
    float a, b, c;
    if (!(ss >> a >> b >> c)) continue;
    x.push_back(a);
    y.push_back(b);
    z.push_back(c);
  }
  out.n = (int64_t)x.size();
  out.add("x") = x;
  out.add("y") = y;
  out.add("z") = z;
  return GS_OK;
}

// ---------------------------------------------------------------- PRNG
struct Xoshiro256ss {
  uint64_t s[4];
  static uint64_t splitmix64(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  explicit Xoshiro256ss(uint64_t seed) {
    uint64_t x = seed;
    for (auto& v : s) v = splitmix64(x);
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t result = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return result;
  }
  double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }  // [0,1)
  double normal() {
    // Box-Muller (one value per pair of draws; deterministic)
    const double u1 = 1.0 - uniform();  // (0,1]
    const double u2 = uniform();
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
};

}  // namespace
}  // namespace gsh

using gsh::set_error;

extern "C" {

int gs_ply_load(const char* path, gs_ply** out) {
  if (!path || !out) {
    set_error("gs_ply_load: null argument");
    return GS_EINVAL;
  }
  auto p = std::make_unique<gs_ply>();
  const std::string s(path);
  int rc;
  // splat::loadPoints (file_io.cpp:44-55): dispatch on the lower-cased extension
  if (gsh::ends_with_ci(s, ".xyz")) {
    rc = gsh::load_xyz(s, *p);
  } else if (gsh::ends_with_ci(s, ".ply")) {
    rc = gsh::load_ply(s, *p);
  } else {
    set_error("Unsupported file extension: " + s);
    return GS_EIO;
  }
  if (rc != GS_OK) return rc;
  *out = p.release();
  return GS_OK;
}

int gs_ply_save(const gs_ply* p, const char* path) {
  if (!p || !path) {
    set_error("gs_ply_save: null argument");
    return GS_EINVAL;
  }
  std::ofstream o(path, std::ios::binary);
  if (!o) {
    set_error(std::string("cannot write ") + path);
    return GS_EIO;
  }
  o << "ply\nformat binary_little_endian 1.0\nelement vertex " << p->n << "\n";
  for (const auto& k : p->order) o << "property float " << k << "\n";
  o << "end_header\n";
  std::vector<const float*> cols;
  for (const auto& k : p->order) cols.push_back(p->props.at(k).data());
  std::vector<float> row(cols.size());
  for (int64_t i = 0; i < p->n; ++i) {
    for (size_t k = 0; k < cols.size(); ++k) row[k] = cols[k][i];
    o.write((const char*)row.data(), (std::streamsize)(row.size() * sizeof(float)));
  }
  if (!o) {
    set_error(std::string("write failed: ") + path);
    return GS_EIO;
  }
  return GS_OK;
}

void gs_ply_free(gs_ply* p) { delete p; }

int64_t gs_ply_count(const gs_ply* p) { return p ? p->n : -1; }

int gs_ply_has(const gs_ply* p, const char* name) {
  return (p && name && p->get(name)) ? 1 : 0;
}

int gs_ply_get(const gs_ply* p, const char* name, float* dst, size_t n) {
  if (!p || !name || !dst) {
    set_error("gs_ply_get: null argument");
    return GS_EINVAL;
  }
  const auto* v = p->get(name);
  if (!v) {
    set_error(std::string("no property ") + name);
    return GS_EINVAL;
  }
  if (n < v->size()) {
    set_error("gs_ply_get: destination too small");
    return GS_EINVAL;
  }
  std::memcpy(dst, v->data(), v->size() * sizeof(float));
  return GS_OK;
}

int gs_synth_params_init(gs_synth_params* sp) {
  if (!sp) return GS_EINVAL;
  std::memset(sp, 0, sizeof(*sp));
  sp->n = 1000000;
  sp->seed = 1;
  sp->sh_degree = 3;
  // point_cloud_12.ply bounds after centring (SURVEY §8 d): ~ +-4.36 x +-3.12 x +-2.58
  const float half[3] = {4.36f, 3.12f, 2.58f};
  for (int i = 0; i < 3; ++i) {
    sp->bb_min[i] = -half[i];
    sp->bb_max[i] = half[i];
  }
  sp->log_scale_mu = -5.6f;  // median radius 4 px at 1080p, fxy[1] = 1 (tools/calibrate_synth.py)
  sp->log_scale_sigma = 0.5f;
  sp->opacity_lo = 0.5f;
  sp->opacity_hi = 8.0f;
  sp->cluster_sigma = 0.02f;
  return GS_OK;
}

int gs_ply_synthetic(const gs_synth_params* sp, gs_ply** out) {
  if (!sp || !out || (sp->sh_degree != 0 && sp->sh_degree != 3)) {
    set_error("gs_ply_synthetic: bad arguments (sh_degree must be 0 or 3)");
    return GS_EINVAL;
  }
  if (sp->n_cluster && !sp->cluster_xyz) {
    set_error("gs_ply_synthetic: n_cluster without cluster_xyz");
    return GS_EINVAL;
  }
  auto p = std::make_unique<gs_ply>();
  p->n = (int64_t)sp->n;
  // INRIA 3DGS vertex layout
  float* x = p->add("x").data();
  float* y = p->add("y").data();
  float* z = p->add("z").data();
  float* nx = p->add("nx").data();
  float* ny = p->add("ny").data();
  float* nz = p->add("nz").data();
  float* dc[3] = {p->add("f_dc_0").data(), p->add("f_dc_1").data(), p->add("f_dc_2").data()};
  std::vector<float*> rest;
  if (sp->sh_degree == 3)
    for (int k = 0; k < 45; ++k) rest.push_back(p->add("f_rest_" + std::to_string(k)).data());
  float* op = p->add("opacity").data();
  float* sc[3] = {p->add("scale_0").data(), p->add("scale_1").data(), p->add("scale_2").data()};
  float* rot[4] = {p->add("rot_0").data(), p->add("rot_1").data(), p->add("rot_2").data(),
                   p->add("rot_3").data()};
  gsh::Xoshiro256ss rng(sp->seed);
  for (int64_t i = 0; i < p->n; ++i) {
    if (sp->n_cluster) {
      const uint64_t j = rng.next() % sp->n_cluster;
      const float* c = sp->cluster_xyz + 3 * j;
      x[i] = c[0] + (float)(sp->cluster_sigma * rng.normal());
      y[i] = c[1] + (float)(sp->cluster_sigma * rng.normal());
      z[i] = c[2] + (float)(sp->cluster_sigma * rng.normal());
    } else {
      x[i] = sp->bb_min[0] + (float)rng.uniform() * (sp->bb_max[0] - sp->bb_min[0]);
      y[i] = sp->bb_min[1] + (float)rng.uniform() * (sp->bb_max[1] - sp->bb_min[1]);
      z[i] = sp->bb_min[2] + (float)rng.uniform() * (sp->bb_max[2] - sp->bb_min[2]);
    }
    nx[i] = ny[i] = nz[i] = 0.0f;
    for (int k = 0; k < 3; ++k)
      sc[k][i] = (float)(sp->log_scale_mu + sp->log_scale_sigma * rng.normal());
    for (int k = 0; k < 4; ++k) rot[k][i] = (float)rng.normal();
    op[i] = (float)(sp->opacity_lo + (sp->opacity_hi - sp->opacity_lo) * rng.uniform());
    for (int k = 0; k < 3; ++k) dc[k][i] = (float)rng.normal();
    for (float* r : rest) r[i] = (float)(0.05 * rng.normal());
  }
  *out = p.release();
  return GS_OK;
}

int gs_scene_prepare(const gs_ply* p, gs_gaussian3d* out, size_t n, float* bb_out) {
  if (!p || !out || n < (size_t)p->n) {
    set_error("gs_scene_prepare: bad arguments");
    return GS_EINVAL;
  }
  const auto *px = p->get("x"), *py = p->get("y"), *pz = p->get("z");
  if (!px || !py || !pz) {
    set_error("gs_scene_prepare: x/y/z missing");
    return GS_EINVAL;
  }
  const int64_t N = p->n;
  std::vector<float> X(*px), Y(*py), Z(*pz);
  // splat::Bounds3f(pts) (geometry.hpp:18-40): std::min / std::max per axis
  auto bounds = [&](float* mn, float* mx) {
    for (int k = 0; k < 3; ++k) {
      mn[k] = std::numeric_limits<float>::infinity();
      mx[k] = -std::numeric_limits<float>::infinity();
    }
    for (int64_t i = 0; i < N; ++i) {
      const float v[3] = {X[i], Y[i], Z[i]};
      for (int k = 0; k < 3; ++k) {
        mn[k] = std::min(mn[k], v[k]);
        mx[k] = std::max(mx[k], v[k]);
      }
    }
  };
  float mn[3], mx[3];
  bounds(mn, mx);
  // splat.cpp:93-100: translate so the centroid is zero, then negate z
  const float centre[3] = {(mx[0] + mn[0]) * 0.5f, (mx[1] + mn[1]) * 0.5f, (mx[2] + mn[2]) * 0.5f};
  for (int64_t i = 0; i < N; ++i) {
    X[i] = X[i] - centre[0];
    Y[i] = Y[i] - centre[1];
    Z[i] = Z[i] - centre[2];
    Z[i] = -Z[i];
  }
  bounds(mn, mx);
  if (bb_out) {
    for (int k = 0; k < 3; ++k) {
      bb_out[k] = mn[k];
      bb_out[3 + k] = mx[k];
    }
  }
  const auto* dc0 = p->get("f_dc_0");
  const auto* dc1 = p->get("f_dc_1");
  const auto* dc2 = p->get("f_dc_2");
  const bool has_dc = dc0 && dc1 && dc2 && !dc0->empty();
  const auto* op = p->get("opacity");
  const auto *s0 = p->get("scale_0"), *s1 = p->get("scale_1"), *s2 = p->get("scale_2");
  const auto *r0 = p->get("rot_0"), *r1 = p->get("rot_1"), *r2 = p->get("rot_2"),
             *r3 = p->get("rot_3");
  if (has_dc && (!op || !s0 || !s1 || !s2 || !r0 || !r1 || !r2 || !r3)) {
    set_error("gs_scene_prepare: incomplete 3DGS properties");
    return GS_EINVAL;
  }
  const float SH_C0 = 0.28209479177387814f;  // splat.cpp:136
  for (int64_t i = 0; i < N; ++i) {
    gs_gaussian3d& g = out[i];
    g.mean[0] = X[i];
    g.mean[1] = Y[i];
    g.mean[2] = Z[i];
    g.mean[3] = 1.0f;
    if (has_dc) {
      float c[3] = {SH_C0 * (*dc0)[i], SH_C0 * (*dc1)[i], SH_C0 * (*dc2)[i]};
      for (int k = 0; k < 3; ++k) {
        c[k] = c[k] + 0.5f;
        c[k] = (c[k] < 0.0f) ? 0.0f : c[k];  // glm::max(colour, vec3(0))
      }
      g.colour[0] = c[0];
      g.colour[1] = c[1];
      g.colour[2] = c[2];
      g.colour[3] = (*op)[i];
      g.scale[0] = (*s0)[i];
      g.scale[1] = (*s1)[i];
      g.scale[2] = (*s2)[i];
      g.rot[0] = (*r0)[i];
      g.rot[1] = (*r1)[i];
      g.rot[2] = (*r2)[i];
      g.rot[3] = (*r3)[i];
    } else {
      // splat.cpp:157-160 (rot is left uninitialised there; identity here)
      g.colour[0] = g.colour[1] = g.colour[2] = 0.05f;
      g.colour[3] = 1.0f;
      g.scale[0] = g.scale[1] = g.scale[2] = 1.0f;
      g.rot[0] = 1.0f;
      g.rot[1] = g.rot[2] = g.rot[3] = 0.0f;
    }
    g.gid = static_cast<float>(i) + 1.0f;  // splat.cpp:161
  }
  return GS_OK;
}

}  // extern "C"
