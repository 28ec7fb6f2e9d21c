// Restart/UMEAN file I/O.  HDF5 is bound at run time with dlopen so that the
// core library does not drag the image's conda runtime into every process; the reference linked
// hdf5/hdf5_hl directly (Makefile:4) and gathered every x-plane on rank 0 with an MPI_Barrier per
// plane (hit_mpi.c:257-339).  Here each rank writes its own planes as hyperslabs of one file.
#include "channel/io.hpp"

#include <dlfcn.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>

#include "channel/common.hpp"

namespace channel {

namespace {
using hid_t = int64_t;
using herr_t = int;
using htri_t = int;
using hsize_t = unsigned long long;

struct H5 {
  void* lib = nullptr;
  herr_t (*open)();
  hid_t (*Fcreate)(const char*, unsigned, hid_t, hid_t);
  hid_t (*Fopen)(const char*, unsigned, hid_t);
  herr_t (*Fclose)(hid_t);
  hid_t (*Screate_simple)(int, const hsize_t*, const hsize_t*);
  hid_t (*Screate)(int);
  herr_t (*Sclose)(hid_t);
  herr_t (*Sselect_hyperslab)(hid_t, int, const hsize_t*, const hsize_t*, const hsize_t*, const hsize_t*);
  int (*Sget_simple_extent_dims)(hid_t, hsize_t*, hsize_t*);
  hid_t (*Dcreate2)(hid_t, const char*, hid_t, hid_t, hid_t, hid_t, hid_t);
  hid_t (*Dopen2)(hid_t, const char*, hid_t);
  herr_t (*Dclose)(hid_t);
  herr_t (*Dwrite)(hid_t, hid_t, hid_t, hid_t, hid_t, const void*);
  herr_t (*Dread)(hid_t, hid_t, hid_t, hid_t, hid_t, void*);
  hid_t (*Dget_space)(hid_t);
  hid_t (*Pcreate)(hid_t);
  herr_t (*Pset_fill_value)(hid_t, hid_t, const void*);
  herr_t (*Pclose)(hid_t);
  hid_t (*Acreate2)(hid_t, const char*, hid_t, hid_t, hid_t, hid_t);
  herr_t (*Awrite)(hid_t, hid_t, const void*);
  herr_t (*Aclose)(hid_t);
  htri_t (*Aexists)(hid_t, const char*);
  hid_t (*Aopen)(hid_t, const char*, hid_t);
  herr_t (*Aread)(hid_t, hid_t, void*);
  herr_t (*Adelete)(hid_t, const char*);
  int (*Aget_num_attrs)(hid_t);
  hid_t (*Aopen_idx)(hid_t, unsigned);
  long (*Aget_name)(hid_t, size_t, char*);
  herr_t (*Eset_auto2)(hid_t, void*, void*);
  hid_t* T_NATIVE_FLOAT = nullptr;
  hid_t* T_NATIVE_DOUBLE = nullptr;
  hid_t* P_DATASET_CREATE = nullptr;
  std::string error;

  template <typename F>
  bool sym(F& f, const char* name) {
    f = reinterpret_cast<F>(dlsym(lib, name));
    if (!f) error = std::string("missing symbol ") + name;
    return f != nullptr;
  }
  H5() {
    const char* env = std::getenv("CHANNEL_HDF5_LIB");
    const char* cands[] = {env, "libhdf5.so.103", "/opt/conda/lib/libhdf5.so.103", "libhdf5.so", "/opt/conda/lib/libhdf5.so"};
    for (const char* c : cands) {
      if (!c) continue;
      lib = dlopen(c, RTLD_NOW | RTLD_LOCAL);
      if (lib) break;
    }
    if (!lib) {
      error = "libhdf5 not found (set CHANNEL_HDF5_LIB)";
      return;
    }
    bool ok = sym(open, "H5open") && sym(Fcreate, "H5Fcreate") && sym(Fopen, "H5Fopen") && sym(Fclose, "H5Fclose") &&
              sym(Screate_simple, "H5Screate_simple") && sym(Screate, "H5Screate") && sym(Sclose, "H5Sclose") &&
              sym(Sselect_hyperslab, "H5Sselect_hyperslab") && sym(Sget_simple_extent_dims, "H5Sget_simple_extent_dims") &&
              sym(Dcreate2, "H5Dcreate2") && sym(Dopen2, "H5Dopen2") && sym(Dclose, "H5Dclose") &&
              sym(Dwrite, "H5Dwrite") && sym(Dread, "H5Dread") && sym(Dget_space, "H5Dget_space") &&
              sym(Pcreate, "H5Pcreate") && sym(Pset_fill_value, "H5Pset_fill_value") && sym(Pclose, "H5Pclose") &&
              sym(Acreate2, "H5Acreate2") && sym(Awrite, "H5Awrite") && sym(Aclose, "H5Aclose") &&
              sym(Aexists, "H5Aexists") && sym(Aopen, "H5Aopen") && sym(Aread, "H5Aread") && sym(Adelete, "H5Adelete") &&
              sym(Aget_num_attrs, "H5Aget_num_attrs") && sym(Aopen_idx, "H5Aopen_idx") && sym(Aget_name, "H5Aget_name") &&
              sym(Eset_auto2, "H5Eset_auto2") && sym(T_NATIVE_FLOAT, "H5T_NATIVE_FLOAT_g") &&
              sym(T_NATIVE_DOUBLE, "H5T_NATIVE_DOUBLE_g") && sym(P_DATASET_CREATE, "H5P_CLS_DATASET_CREATE_ID_g");
    if (!ok) {
      dlclose(lib);
      lib = nullptr;
      return;
    }
    open();
    Eset_auto2(0, nullptr, nullptr);
  }
};

H5& h5raw() {
  static H5 inst;
  return inst;
}
H5& h5() {
  H5& inst = h5raw();
  CH_CHECK(inst.lib, "HDF5 unavailable: " << inst.error);
  return inst;
}

constexpr unsigned ACC_RDONLY = 0x0000u, ACC_RDWR = 0x0001u, ACC_TRUNC = 0x0002u;
constexpr hid_t P_DEFAULT = 0, S_ALL = 0;
constexpr int S_SELECT_SET = 0, S_SCALAR = 0;

struct Hid {
  hid_t id;
  herr_t (*close)(hid_t);
  Hid(hid_t i, herr_t (*c)(hid_t), const std::string& what) : id(i), close(c) {
    CH_CHECK(i >= 0, "HDF5: " << what << " failed");
  }
  ~Hid() {
    if (id >= 0) close(id);
  }
};
}  // namespace

bool hdf5_available() { return h5raw().lib != nullptr; }

void h5_create_field(const std::string& path, int NX, int NY, int NZ, bool fp64, int Kx) {
  H5& h = h5();
  Hid f(h.Fcreate(path.c_str(), ACC_TRUNC, P_DEFAULT, P_DEFAULT), h.Fclose, "create " + path);
  const hsize_t dims[3] = {static_cast<hsize_t>(NX), static_cast<hsize_t>(NY), static_cast<hsize_t>(2 * NZ)};
  Hid sp(h.Screate_simple(3, dims, nullptr), h.Sclose, "dataspace");
  Hid pl(h.Pcreate(*h.P_DATASET_CREATE), h.Pclose, "dcpl");
  const double zero = 0.0;
  h.Pset_fill_value(pl.id, *h.T_NATIVE_DOUBLE, &zero);
  Hid d(h.Dcreate2(f.id, "u", fp64 ? *h.T_NATIVE_DOUBLE : *h.T_NATIVE_FLOAT, sp.id, P_DEFAULT, pl.id, P_DEFAULT),
        h.Dclose, "create dataset u");
  // explicitly write the zero planes nobody else writes (all of them when Kx < 0)
  std::vector<float> zp(static_cast<size_t>(NY) * 2 * NZ, 0.0f);
  for (int i = 0; i < NX; ++i) {
    const int kx = i < NX / 2 ? i : i - NX;  // FFT order
    if (Kx >= 0 && kx >= -Kx && kx <= Kx) continue;
    const hsize_t start[3] = {static_cast<hsize_t>(i), 0, 0};
    const hsize_t count[3] = {1, static_cast<hsize_t>(NY), static_cast<hsize_t>(2 * NZ)};
    Hid fs(h.Dget_space(d.id), h.Sclose, "filespace");
    h.Sselect_hyperslab(fs.id, S_SELECT_SET, start, nullptr, count, nullptr);
    Hid ms(h.Screate_simple(3, count, nullptr), h.Sclose, "memspace");
    CH_CHECK(h.Dwrite(d.id, *h.T_NATIVE_FLOAT, ms.id, fs.id, P_DEFAULT, zp.data()) >= 0, "HDF5 write zero plane");
  }
}

void h5_write_planes(const std::string& path, const std::vector<int>& planes, const std::vector<double>& data) {
  H5& h = h5();
  Hid f(h.Fopen(path.c_str(), ACC_RDWR, P_DEFAULT), h.Fclose, "open " + path);
  Hid d(h.Dopen2(f.id, "u", P_DEFAULT), h.Dclose, "open dataset u");
  hsize_t dims[3];
  {
    Hid fs(h.Dget_space(d.id), h.Sclose, "filespace");
    h.Sget_simple_extent_dims(fs.id, dims, nullptr);
  }
  const size_t plane = static_cast<size_t>(dims[1] * dims[2]);
  CH_CHECK(data.size() == plane * planes.size(), "h5_write_planes: size mismatch");
  for (size_t k = 0; k < planes.size(); ++k) {
    const hsize_t start[3] = {static_cast<hsize_t>(planes[k]), 0, 0};
    const hsize_t count[3] = {1, dims[1], dims[2]};
    Hid fs(h.Dget_space(d.id), h.Sclose, "filespace");
    h.Sselect_hyperslab(fs.id, S_SELECT_SET, start, nullptr, count, nullptr);
    Hid ms(h.Screate_simple(3, count, nullptr), h.Sclose, "memspace");
    CH_CHECK(h.Dwrite(d.id, *h.T_NATIVE_DOUBLE, ms.id, fs.id, P_DEFAULT, data.data() + k * plane) >= 0,
             "HDF5 write plane " << planes[k]);
  }
}

void h5_read_planes(const std::string& path, const std::vector<int>& planes, std::vector<double>& data, int dims_out[3]) {
  H5& h = h5();
  Hid f(h.Fopen(path.c_str(), ACC_RDONLY, P_DEFAULT), h.Fclose, "open " + path);
  Hid d(h.Dopen2(f.id, "u", P_DEFAULT), h.Dclose, "open dataset u");
  hsize_t dims[3];
  {
    Hid fs(h.Dget_space(d.id), h.Sclose, "filespace");
    CH_CHECK(h.Sget_simple_extent_dims(fs.id, dims, nullptr) == 3, "dataset u is not 3-D");
  }
  for (int i = 0; i < 3; ++i) dims_out[i] = static_cast<int>(dims[i]);
  const size_t plane = static_cast<size_t>(dims[1] * dims[2]);
  data.assign(plane * planes.size(), 0.0);
  for (size_t k = 0; k < planes.size(); ++k) {
    CH_CHECK(planes[k] < static_cast<int>(dims[0]), "plane index out of range");
    const hsize_t start[3] = {static_cast<hsize_t>(planes[k]), 0, 0};
    const hsize_t count[3] = {1, dims[1], dims[2]};
    Hid fs(h.Dget_space(d.id), h.Sclose, "filespace");
    h.Sselect_hyperslab(fs.id, S_SELECT_SET, start, nullptr, count, nullptr);
    Hid ms(h.Screate_simple(3, count, nullptr), h.Sclose, "memspace");
    CH_CHECK(h.Dread(d.id, *h.T_NATIVE_DOUBLE, ms.id, fs.id, P_DEFAULT, data.data() + k * plane) >= 0,
             "HDF5 read plane " << planes[k]);
  }
}

void h5_write_attrs(const std::string& path, const std::map<std::string, double>& attrs) {
  H5& h = h5();
  Hid f(h.Fopen(path.c_str(), ACC_RDWR, P_DEFAULT), h.Fclose, "open " + path);
  for (const auto& kv : attrs) {
    if (h.Aexists(f.id, kv.first.c_str()) > 0) h.Adelete(f.id, kv.first.c_str());
    Hid sp(h.Screate(S_SCALAR), h.Sclose, "scalar space");
    Hid a(h.Acreate2(f.id, kv.first.c_str(), *h.T_NATIVE_DOUBLE, sp.id, P_DEFAULT, P_DEFAULT), h.Aclose,
          "attribute " + kv.first);
    h.Awrite(a.id, *h.T_NATIVE_DOUBLE, &kv.second);
  }
}

std::map<std::string, double> h5_read_attrs(const std::string& path) {
  H5& h = h5();
  std::map<std::string, double> out;
  Hid f(h.Fopen(path.c_str(), ACC_RDONLY, P_DEFAULT), h.Fclose, "open " + path);
  static const char* keys[] = {"time", "dt", "step", "Re", "Q", "LX", "LZ", "NX", "NY", "NZ", "format_version"};
  for (const char* k : keys) {
    if (h.Aexists(f.id, k) <= 0) continue;
    Hid a(h.Aopen(f.id, k, P_DEFAULT), h.Aclose, std::string("attribute ") + k);
    double v = 0;
    if (h.Aread(a.id, *h.T_NATIVE_DOUBLE, &v) >= 0) out[k] = v;
  }
  return out;
}

void h5_write_vector(const std::string& path, const std::string& name, const std::vector<double>& v) {
  H5& h = h5();
  Hid f(h.Fopen(path.c_str(), ACC_RDWR, P_DEFAULT), h.Fclose, "open " + path);
  const hsize_t dims[1] = {static_cast<hsize_t>(v.size())};
  Hid sp(h.Screate_simple(1, dims, nullptr), h.Sclose, "dataspace");
  Hid d(h.Dcreate2(f.id, name.c_str(), *h.T_NATIVE_DOUBLE, sp.id, P_DEFAULT, P_DEFAULT, P_DEFAULT), h.Dclose,
        "create dataset " + name);
  CH_CHECK(h.Dwrite(d.id, *h.T_NATIVE_DOUBLE, S_ALL, S_ALL, P_DEFAULT, v.data()) >= 0, "HDF5 write " << name);
}

bool h5_read_vector(const std::string& path, const std::string& name, std::vector<double>& v) {
  H5& h = h5();
  Hid f(h.Fopen(path.c_str(), ACC_RDONLY, P_DEFAULT), h.Fclose, "open " + path);
  const hid_t did = h.Dopen2(f.id, name.c_str(), P_DEFAULT);
  if (did < 0) return false;
  Hid d(did, h.Dclose, "open dataset " + name);
  hsize_t dims[1] = {0};
  {
    Hid fs(h.Dget_space(d.id), h.Sclose, "filespace");
    CH_CHECK(h.Sget_simple_extent_dims(fs.id, dims, nullptr) == 1, "dataset " << name << " is not 1-D");
  }
  v.assign(dims[0], 0.0);
  CH_CHECK(h.Dread(d.id, *h.T_NATIVE_DOUBLE, S_ALL, S_ALL, P_DEFAULT, v.data()) >= 0, "HDF5 read " << name);
  return true;
}

void umean_write(const std::string& path, const std::vector<double>& U) {
  std::ofstream f(path, std::ios::binary | std::ios::trunc);
  CH_CHECK(f.good(), "cannot write " << path);
  for (double u : U) {
    const float rec[2] = {static_cast<float>(u), 0.0f};
    f.write(reinterpret_cast<const char*>(rec), sizeof(rec));
  }
}

std::vector<double> umean_read(const std::string& path, int NY) {
  std::ifstream f(path, std::ios::binary);
  CH_CHECK(f.good(), "cannot read " << path);
  std::vector<double> U(NY);
  for (int j = 0; j < NY; ++j) {
    float rec[2];
    f.read(reinterpret_cast<char*>(rec), sizeof(rec));
    CH_CHECK(f.good(), "UMEAN file " << path << " too short");
    U[j] = rec[0];
  }
  return U;
}

}  // namespace channel
