// Restart and statistics file I/O, byte-compatible with the reference.
//
//  * G / DDV: HDF5, one dataset "u", H5T_NATIVE_FLOAT, declared dims {NX, NY, 2*NZ}, holding for
//    each global kx plane i (FFT order) the values in [kz][y][re,im] order, in "N2 units"
//    (stored = NX*(2NZ-2) * Fourier coefficient) (hit_mpi.c:257-422, io.c:3-72).
//    We add root-group attributes (time, dt, step, Re, ...) that old readers ignore.
//  * UMEAN: raw NY records of {float U*N2, float 0} (meanUevol.c:153-176).
// HDF5 is loaded at run time (dlopen of the image's libhdf5) so the core library has no hard
// dependency on it; a missing libhdf5 makes restart I/O fail loudly.
#pragma once

#include <map>
#include <string>
#include <vector>

namespace channel {

bool hdf5_available();

// Create (truncate) a restart file with a zero-filled dataset "u" {NX, NY, 2NZ} (float32, or
// float64 for fp64 storage).  Unwritten data reads as the fill value 0; with Kx >= 0 the planes of
// the dealiased kx (|kx| > Kx, which no rank writes) are also written explicitly as zeros, so the
// file is fully defined for readers that ignore fill values while the retained planes (written by
// their owners) are written only once.  Kx < 0: every plane is zero-written.
void h5_create_field(const std::string& path, int NX, int NY, int NZ, bool fp64, int Kx = -1);
// Write planes (each NY*2NZ values in [kz][y][re,im] order) at the given global plane indices.
void h5_write_planes(const std::string& path, const std::vector<int>& planes, const std::vector<double>& data);
// Read planes; also returns the dataset dims.
void h5_read_planes(const std::string& path, const std::vector<int>& planes, std::vector<double>& data, int dims[3]);
void h5_write_attrs(const std::string& path, const std::map<std::string, double>& attrs);
std::map<std::string, double> h5_read_attrs(const std::string& path);

// extra 1-D float64 dataset (e.g. "umean": U(y) at full precision next to "u"; old readers ignore it)
void h5_write_vector(const std::string& path, const std::string& name, const std::vector<double>& v);
bool h5_read_vector(const std::string& path, const std::string& name, std::vector<double>& v);  // false: absent

void umean_write(const std::string& path, const std::vector<double>& U_times_N2);
std::vector<double> umean_read(const std::string& path, int NY);

}  // namespace channel
