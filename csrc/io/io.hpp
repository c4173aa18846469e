// heat3d-mi355x — output and persistence.
//
// Tecplot ASCII writer byte-compatible with the reference's output/out.dat
// (heat3D.cu:1109-1179): TITLE / VARIABLES / one ZONE per
// rank, rows of "%15.5e" columns (plus "%5d" rank when P > 1), k outermost and
// i innermost.  The reference wrote it serially on rank 0 after an MPI gather
// and silently produced nothing when output/ was missing; here the
// directory is created and lines are formatted in parallel.
//
// Checkpoints (new — the reference has no restart): a directory
// with meta.json and field.raw, the full N0 x N1 x N2 grid in the run's dtype,
// z fastest.  Every process pwrite()s its own extended box, so the file is
// independent of the decomposition and a run can restart on a different
// number of ranks.
#pragma once

#include <array>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "../core/common.hpp"

namespace heat3d {
namespace io {

struct Zone {
  int rank = 0;        // value of the rank column
  int title = 0;       // ZONE T = "<title>"
  int64_t lo[3] = {0, 0, 0};  // global vertex box [lo, hi)
  int64_t hi[3] = {0, 0, 0};
};

// `field` is the global grid (N0*N1*N2 doubles, z fastest).
void write_tecplot(const std::string& path, const std::vector<double>& field, const int64_t N[3],
                   const double h[3], const std::vector<Zone>& zones, bool rank_column);

void make_dirs(const std::string& path);
std::string dirname_of(const std::string& path);

// Minimal flat JSON object (string/number/bool/array-of-number values).
class Json {
 public:
  void set(const std::string& k, const std::string& v);
  void set(const std::string& k, double v);
  void set(const std::string& k, int64_t v);
  void set_bool(const std::string& k, bool v);
  void set_raw(const std::string& k, const std::string& raw);
  std::string dump() const;
  static std::map<std::string, std::string> parse_flat(const std::string& text);

 private:
  std::vector<std::pair<std::string, std::string>> kv_;
};

std::string read_file(const std::string& path);
void write_file_atomic(const std::string& path, const std::string& content);

// Raw global-grid file access (positioned I/O, any process, disjoint ranges).
// truncate = create / empty the file (one process, before the others open it).
int open_raw(const std::string& path, bool write, bool truncate = false);
void truncate_raw(int fd, int64_t size);
void fsync_raw(int fd);
int64_t file_size(const std::string& path);  // -1 if missing
// rename + fsync of the directory entry
void rename_durable(const std::string& from, const std::string& to);
std::vector<std::string> list_dir(const std::string& dir);
void remove_file(const std::string& path);
void pwrite_all(int fd, const void* p, std::size_t n, int64_t off);
void pread_all(int fd, void* p, std::size_t n, int64_t off);
void close_raw(int fd);

}  // namespace io
}  // namespace heat3d
