// ref_ply_dump.cpp -- TEST INFRASTRUCTURE ONLY (never linked into or called
// by libgsplat.so).  Reads a .ply with the reference's own vendored PLY parser
// (happly.h, compiled from where it lies: /root/reference/include/happly.h)
// through the same calls as splat::fillPlyProperties
// (/root/reference/src/splat/file_io.cpp:57-77: getElement("vertex")
// .getProperty<float>(name) for the 14 3DGS properties), and writes them as
// raw float32: n (int64) then the 14 arrays in that order.  The reference's
// file_io.cpp itself needs glm (an empty submodule here), so this driver
// restates its two-line fillProperty; the parsing is happly's.
// Used by tests/test_ref_ply.py to pin the product's PLY reader
// (gs_ply_load, csrc/host/gs_scene.cpp) to the reference's parser.
#include <happly.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: ref_ply_dump <in.ply> <out.bin>\n");
    return 2;
  }
  static const char* kProps[14] = {"x",       "y",       "z",       "f_dc_0",  "f_dc_1",
                                   "f_dc_2",  "opacity", "scale_0", "scale_1", "scale_2",
                                   "rot_0",   "rot_1",   "rot_2",   "rot_3"};
  try {
    happly::PLYData ply(argv[1]);
    std::vector<std::vector<float>> cols;
    for (const char* p : kProps) cols.push_back(ply.getElement("vertex").getProperty<float>(p));
    std::FILE* f = std::fopen(argv[2], "wb");
    if (!f) return 1;
    const int64_t n = (int64_t)cols[0].size();
    std::fwrite(&n, sizeof(n), 1, f);
    for (const auto& c : cols) std::fwrite(c.data(), sizeof(float), c.size(), f);
    std::fclose(f);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "ref_ply_dump: %s\n", e.what());
    return 1;
  }
  return 0;
}
