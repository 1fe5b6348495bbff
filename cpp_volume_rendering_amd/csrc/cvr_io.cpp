// cvr_io.cpp — native readers for the reference's input formats.  The
// reference readers are MSVC-only (fopen_s, sscanf_s, `unsigned char(v)` casts:
// libs/file_utils/rawloader.cpp:16, libs/volvis_utils/reader.cpp:317,352), so
// they are re-implemented here with the same grammar and semantics.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/cvr.h"

namespace {

std::string basename_of(const std::string& p) {
  size_t a = p.find_last_of("/\\");
  return a == std::string::npos ? p : p.substr(a + 1);
}

// ---------------------------------------------------------------------------
// PVM / DDS (the V^3 volume format of libs/file_utils/pvm.cpp:191-620).  A .pvm
// file is either plain or a "Differential Data Stream": an 8-byte id ("DDS v3d\n",
// or "DDS v3e\n" = interleaved in blocks of 2^24 bytes) and a bit stream of
// big-endian 32-bit words, MSB first.  The stream holds 2 bits (skip - 1),
// 16 bits (strip - 1), then runs: 7 bits run length (0 ends the stream), 3 bits
// code -> bits per delta (code >= 1 ? code + 1 : code), and `run` deltas of
// that many bits biased by 2^bits / 2.  A delta adds to the running byte value
// (mod 256), plus, past the first `strip` bytes (strip > 1), the difference of
// the two bytes one `strip` earlier.  The bytes are then re-interleaved with
// stride `skip` (DDS_interleave).  The payload is the PVM text header, the
// voxels and (PVM3) four strings.
// ---------------------------------------------------------------------------
struct DdsBits {
  const unsigned char* data;
  size_t size, pos = 0;        // size padded to whole words, zeros past the end
  uint32_t buffer = 0;
  uint32_t bufsize = 0;
  static uint32_t shl(uint32_t v, uint32_t b) { return b >= 32 ? 0u : v << b; }
  static uint32_t shr(uint32_t v, uint32_t b) { return b >= 32 ? 0u : v >> b; }
  uint32_t read(uint32_t bits) {
    uint32_t value;
    if (bits < bufsize) {
      bufsize -= bits;
      value = shr(buffer, bufsize);
    } else {
      value = shl(buffer, bits - bufsize);
      if (pos >= size) {
        buffer = 0;
      } else {
        buffer = (uint32_t)data[pos] << 24 | (uint32_t)data[pos + 1] << 16 |
                 (uint32_t)data[pos + 2] << 8 | (uint32_t)data[pos + 3];
        pos += 4;
      }
      bufsize += 32 - bits;
      value |= shr(buffer, bufsize);
    }
    buffer &= shl(1, bufsize) - 1;
    return value;
  }
};

// DDS_deinterleave(..., restore = true): undo the encoder's stride-`skip` split,
// whole or per block of skip*block bytes.
void dds_interleave(std::vector<unsigned char>& d, size_t skip, size_t block) {
  if (skip <= 1) return;
  const size_t bytes = d.size();
  auto run = [&](size_t off, size_t len) {
    std::vector<unsigned char> t(len);
    size_t p = off;
    for (size_t i = 0; i < skip; i++)
      for (size_t j = i; j < len; j += skip) t[j] = d[p++];
    std::memcpy(&d[off], t.data(), len);
  };
  if (block == 0) {
    run(0, bytes);
    return;
  }
  size_t k = 0;
  for (; k < bytes / skip / block; k++) run(k * skip * block, skip * block);
  if (bytes > k * skip * block) run(k * skip * block, bytes - k * skip * block);
}

bool dds_decode(std::vector<unsigned char> chunk, size_t block, std::vector<unsigned char>& out) {
  chunk.resize((chunk.size() + 3) / 4 * 4 + 4, 0);
  DdsBits b{chunk.data(), chunk.size() - 4};
  const size_t skip = b.read(2) + 1;
  const size_t strip = b.read(16) + 1;
  out.clear();
  int act = 0;
  for (;;) {
    const uint32_t run = b.read(7);                   // DDS_RL
    if (run == 0) break;
    const uint32_t code = b.read(3);
    const uint32_t bits = code >= 1 ? code + 1 : code;
    for (uint32_t k = 0; k < run; k++) {
      const size_t cnt = out.size();
      if (strip == 1 || cnt <= strip)
        act += (int)b.read(bits) - (int)((1u << bits) / 2);
      else
        act += (int)out[cnt - strip] - (int)out[cnt - strip - 1] + (int)b.read(bits) -
               (int)((1u << bits) / 2);
      while (act < 0) act += 256;
      while (act > 255) act -= 256;
      out.push_back((unsigned char)act);
      if (out.size() > ((size_t)1 << 36)) return false;   // corrupt stream
    }
  }
  dds_interleave(out, skip, block);
  return true;
}

bool read_file(const char* path, std::vector<unsigned char>& buf) {
  FILE* fp = std::fopen(path, "rb");
  if (!fp) return false;
  buf.clear();
  unsigned char tmp[1 << 16];
  size_t n;
  while ((n = std::fread(tmp, 1, sizeof(tmp), fp)) > 0) buf.insert(buf.end(), tmp, tmp + n);
  std::fclose(fp);
  return true;
}

struct Pvm {
  int w = 0, h = 0, d = 0, comps = 0;
  float scale[3] = {1.f, 1.f, 1.f};
  std::vector<unsigned char> payload;
  size_t data_off = 0;
};

// DDSV3::readPVMvolume (pvm.cpp:191-308) minus the description strings
bool read_pvm(const char* path, Pvm& v) {
  std::vector<unsigned char> file;
  if (!read_file(path, file) || file.empty()) return false;
  static const char kV3d[] = "DDS v3d\n", kV3e[] = "DDS v3e\n";
  if (file.size() >= 8 && (!std::memcmp(file.data(), kV3d, 8) || !std::memcmp(file.data(), kV3e, 8))) {
    const bool v3e = !std::memcmp(file.data(), kV3e, 8);
    std::vector<unsigned char> chunk(file.begin() + 8, file.end());
    if (chunk.empty() || !dds_decode(std::move(chunk), v3e ? ((size_t)1 << 24) : 0, v.payload))
      return false;
  } else {
    v.payload.swap(file);                                // readRAWfile: uncompressed
  }
  std::vector<unsigned char>& p = v.payload;
  if (p.size() < 5) return false;
  p.push_back(0);                                        // the reader's '\0' guard
  const char* c = (const char*)p.data();
  int version = 1;
  const char* q;
  if (!std::strncmp(c, "PVM\n", 4)) {
    q = c + 4;
    while (*q == '#')
      while (*q && *q++ != '\n') {}
    if (std::sscanf(q, "%d %d %d", &v.w, &v.h, &v.d) != 3) return false;
  } else {
    if (!std::strncmp(c, "PVM2\n", 5)) version = 2;
    else if (!std::strncmp(c, "PVM3\n", 5)) version = 3;
    else return false;
    q = c + 5;
    if (std::sscanf(q, "%d %d %d\n%g %g %g", &v.w, &v.h, &v.d, &v.scale[0], &v.scale[1],
                    &v.scale[2]) != 6)
      return false;
    if (!(v.scale[0] > 0.f && v.scale[1] > 0.f && v.scale[2] > 0.f)) return false;
    q = std::strchr(q, '\n');
    if (!q) return false;
    q++;
  }
  if (v.w < 1 || v.h < 1 || v.d < 1) return false;
  q = std::strchr(q, '\n');                               // past the dims (v1) / scale (v2, v3)
  if (!q) return false;
  q++;
  if (std::sscanf(q, "%d", &v.comps) != 1 || v.comps < 1) return false;
  q = std::strchr(q, '\n');
  if (!q) return false;
  q++;
  v.data_off = (size_t)(q - c);
  const size_t need = (size_t)v.w * v.h * v.d * v.comps;
  const size_t have = p.size() - 1 - v.data_off;
  if (version == 3 ? have < need : have != need) return false;
  return true;
}

}  // namespace

extern "C" {
#pragma GCC visibility push(default)

// TransferFunctionReader::readtf1d (reader.cpp:744-814)
cvr_status cvr_read_tf1d(const char* path, float* out_rgbt, int* out_n) {
  if (!path || !out_n) return CVR_ERR_ARG;
  std::ifstream f(path);
  if (!f.is_open()) return CVR_ERR_IO;
  std::string interpolation;
  std::getline(f, interpolation);     // "linear" (cubic is never implemented)
  int init = 0;
  if (!(f >> init)) return CVR_ERR_IO;
  int max_density = 255, extuse = 0;
  if (init == 2) {
    if (!(f >> max_density >> extuse)) return CVR_ERR_IO;
  } else if (init == 1) {
    if (!(f >> max_density)) return CVR_ERR_IO;
  }
  int n_rgb = 0;
  if (!(f >> n_rgb) || n_rgb < 0) return CVR_ERR_IO;
  std::vector<double> rgb((size_t)n_rgb * 4);
  for (int i = 0; i < n_rgb; i++) {
    double r, g, b;
    int iso;
    if (!(f >> r >> g >> b >> iso)) return CVR_ERR_IO;
    rgb[i * 4 + 0] = r; rgb[i * 4 + 1] = g; rgb[i * 4 + 2] = b; rgb[i * 4 + 3] = iso;
  }
  int n_a = 0;
  if (!(f >> n_a) || n_a < 0) return CVR_ERR_IO;
  std::vector<double> a((size_t)n_a * 2);
  for (int i = 0; i < n_a; i++) {
    double av;
    int iso;
    if (!(f >> av >> iso)) return CVR_ERR_IO;
    a[i * 2 + 0] = av; a[i * 2 + 1] = iso;
  }
  *out_n = max_density + 1;
  if (!out_rgbt) return CVR_OK;
  return cvr_tf1d_build_rgbt(rgb.data(), n_rgb, a.data(), n_a, max_density, extuse == 1,
                             out_rgbt);
}

// VolumeReader::readraw (reader.cpp:162-225): "name.<bytes>.<W>x<H>x<D>.raw"
cvr_status cvr_read_raw(const char* path, void* voxels, size_t capacity, int* out_w, int* out_h,
                        int* out_d, int* out_bpv) {
  if (!path || !out_w || !out_h || !out_d || !out_bpv) return CVR_ERR_ARG;
  std::string name = basename_of(path);
  size_t ext = name.find_last_of('.');
  if (ext == std::string::npos) return CVR_ERR_IO;
  name = name.substr(0, ext);
  size_t ds = name.find_last_of('.');
  if (ds == std::string::npos) return CVR_ERR_IO;
  std::string sizes = name.substr(ds + 1);
  name = name.substr(0, ds);
  size_t db = name.find_last_of('.');
  std::string bytes = db == std::string::npos ? name : name.substr(db + 1);
  int w = 0, h = 0, d = 0;
  if (std::sscanf(sizes.c_str(), "%dx%dx%d", &w, &h, &d) != 3) return CVR_ERR_IO;
  int bpv = std::atoi(bytes.c_str());
  if (w < 1 || h < 1 || d < 1 || (bpv != 1 && bpv != 2)) return CVR_ERR_IO;
  *out_w = w; *out_h = h; *out_d = d; *out_bpv = bpv;
  if (!voxels) return CVR_OK;
  size_t need = (size_t)w * h * d * bpv;
  if (capacity < need) return CVR_ERR_ARG;
  FILE* fp = std::fopen(path, "rb");
  if (!fp) return CVR_ERR_IO;
  size_t got = std::fread(voxels, 1, need, fp);
  std::fclose(fp);
  return got == need ? CVR_OK : CVR_ERR_IO;
}

// VolumeReader::readsyn (reader.cpp:283-371).  The reference leaves unlisted
// voxels uninitialised (:301); here they are zero.
cvr_status cvr_read_syn(const char* path, uint8_t* voxels, size_t capacity, int* out_w,
                        int* out_h, int* out_d) {
  if (!path || !out_w || !out_h || !out_d) return CVR_ERR_ARG;
  std::ifstream f(path);
  if (!f.is_open()) return CVR_ERR_IO;
  int w, h, d;
  if (!(f >> w >> h >> d) || w < 1 || h < 1 || d < 1) return CVR_ERR_IO;
  *out_w = w; *out_h = h; *out_d = d;
  if (!voxels) return CVR_OK;
  size_t need = (size_t)w * h * d;
  if (capacity < need) return CVR_ERR_ARG;
  std::memset(voxels, 0, need);
  int kind;
  while (f >> kind) {
    if (kind == 1) {
      int x0, y0, z0, x1, y1, z1, v;
      if (!(f >> x0 >> y0 >> z0 >> x1 >> y1 >> z1 >> v)) return CVR_ERR_IO;
      for (int x = x0; x < x1; x++)
        for (int y = y0; y < y1; y++)
          for (int z = z0; z < z1; z++) {
            if (x < 0 || y < 0 || z < 0 || x >= w || y >= h || z >= d) return CVR_ERR_IO;
            voxels[(size_t)x + (size_t)w * y + (size_t)w * h * z] = (uint8_t)v;
          }
    } else {
      int x, y, z, v;
      if (!(f >> x >> y >> z >> v)) return CVR_ERR_IO;
      if (x < 0 || y < 0 || z < 0 || x >= w || y >= h || z >= d) return CVR_ERR_IO;
      voxels[(size_t)x + (size_t)w * y + (size_t)w * h * z] = (uint8_t)v;
    }
  }
  return CVR_OK;
}

// CameraStateList::ReadCameraStates (camerastatelist.cpp:26-87)
cvr_status cvr_read_camera_state(const char* path, int index, cvr_camera* out_cam, char* out_name,
                                 int name_capacity, int* out_count) {
  if (!path) return CVR_ERR_ARG;
  std::ifstream f(path);
  if (!f.is_open()) return CVR_ERR_IO;
  struct State { std::string name; float eye[3], center[3], up[3]; };
  std::vector<State> states;
  std::string line;
  while (!f.eof()) {
    State s{};
    line.clear();
    std::getline(f, line);
    if (!line.empty() && line.back() == '\r') line.pop_back();
    s.name = line;
    line.clear();
    std::getline(f, line);
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line == "ARCBALL") {
      f >> s.eye[0] >> s.eye[1] >> s.eye[2];
      f >> s.center[0] >> s.center[1] >> s.center[2];
      f >> s.up[0] >> s.up[1] >> s.up[2];
      std::getline(f, line);
    }
    states.push_back(s);
  }
  if (out_count) *out_count = (int)states.size();
  if (!out_cam) return CVR_OK;
  if (index < 0 || index >= (int)states.size()) return CVR_ERR_ARG;
  const State& s = states[index];
  for (int i = 0; i < 3; i++) {
    out_cam->eye[i] = s.eye[i];
    out_cam->center[i] = s.center[i];
    out_cam->up[i] = s.up[i];
  }
  out_cam->fovy_deg = 45.0f;   // CameraData default, camera.cpp:25,44
  out_cam->aspect = 0.0f;      // derived from the viewport
  if (out_name && name_capacity > 0) {
    std::strncpy(out_name, s.name.c_str(), (size_t)name_capacity - 1);
    out_name[name_capacity - 1] = 0;
  }
  return CVR_OK;
}

// LightSourceList::ReadLightSourceLists (lightsourcelist.cpp:81-148)
cvr_status cvr_read_light(const char* path, int list, int light, cvr_light* out,
                          int* out_count) {
  if (!path) return CVR_ERR_ARG;
  std::ifstream f(path);
  if (!f.is_open()) return CVR_ERR_IO;
  std::vector<std::vector<std::vector<float>>> lists;
  std::string line;
  while (!f.eof()) {
    line.clear();
    std::getline(f, line);
    int n = 0;
    std::vector<std::vector<float>> lights;
    if (f >> n) {
      for (int i = 0; i < n; i++) {
        std::vector<float> v(13);
        for (int k = 0; k < 13; k++) f >> v[k];
        line.clear();
        std::getline(f, line);
        lights.push_back(v);
      }
    }
    lists.push_back(lights);
  }
  if (out_count) *out_count = (int)lists.size();
  if (!out) return CVR_OK;
  if (list < 0 || list >= (int)lists.size() || light < 0 || light >= (int)lists[list].size())
    return CVR_ERR_ARG;
  const std::vector<float>& v = lists[list][light];
  // position, forward (stored as z_axis = -forward and read back negated), up, right, angle
  for (int i = 0; i < 3; i++) {
    out->position[i] = v[i];
    out->forward[i] = v[3 + i];
    out->up[i] = v[6 + i];
    out->right[i] = v[9 + i];
  }
  out->spot_angle_deg = v[12];
  return CVR_OK;
}

cvr_status cvr_read_light_position(const char* path, int list, int light, float out_pos[3],
                                   int* out_count) {
  cvr_light l;
  cvr_status st = cvr_read_light(path, list, light, out_pos ? &l : nullptr, out_count);
  if (st == CVR_OK && out_pos)
    for (int i = 0; i < 3; i++) out_pos[i] = l.position[i];
  return st;
}

// VolumeReader::readpvm + Pvm::PostProcessData (reader.cpp:100-159,
// pvm.cpp:23-109): 1 component -> u8, 2 components -> u16 assembled as
// data[2i] + 256 * data[2i+1] (the reference's byte order); more components are
// not a scalar volume (CVR_ERR_IO).  scale receives the PVM2/3 voxel spacing
// (1, 1, 1 for PVM1).  Pass voxels = NULL to query the dimensions.
cvr_status cvr_read_pvm(const char* path, void* voxels, size_t capacity, int* out_w, int* out_h,
                        int* out_d, int* out_bpv, float out_scale[3]) {
  if (!path || !out_w || !out_h || !out_d || !out_bpv) return CVR_ERR_ARG;
  Pvm v;
  if (!read_pvm(path, v) || v.comps > 2) return CVR_ERR_IO;
  *out_w = v.w; *out_h = v.h; *out_d = v.d; *out_bpv = v.comps;
  if (out_scale)
    for (int i = 0; i < 3; i++) out_scale[i] = v.scale[i];
  if (!voxels) return CVR_OK;
  const size_t n = (size_t)v.w * v.h * v.d;
  if (capacity < n * v.comps) return CVR_ERR_ARG;
  const unsigned char* src = v.payload.data() + v.data_off;
  if (v.comps == 1) {
    std::memcpy(voxels, src, n);
  } else {
    uint16_t* o = static_cast<uint16_t*>(voxels);
    for (size_t i = 0; i < n; i++) o[i] = (uint16_t)(src[2 * i] + 256u * src[2 * i + 1]);
  }
  return CVR_OK;
}

#pragma GCC visibility pop
}  // extern "C"
