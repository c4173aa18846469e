#include "io.hpp"

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

namespace heat3d {
namespace io {

void make_dirs(const std::string& path) {
  if (path.empty()) return;
  std::string cur;
  std::stringstream ss(path);
  std::string part;
  if (path[0] == '/') cur = "/";
  while (std::getline(ss, part, '/')) {
    if (part.empty()) continue;
    cur += part;
    if (mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST)
      HEAT3D_THROW("mkdir(" << cur << ") failed: " << std::strerror(errno));
    cur += "/";
  }
}

std::string dirname_of(const std::string& path) {
  auto p = path.rfind('/');
  if (p == std::string::npos) return "";
  return path.substr(0, p);
}

// Format "%15.5e" — same bytes as iostream scientific/setprecision(5)/setw(15).
static inline int fmt_e(char* out, double v) { return std::snprintf(out, 32, "%15.5e", v); }

void write_tecplot(const std::string& path, const std::vector<double>& field, const int64_t N[3],
                   const double h[3], const std::vector<Zone>& zones, bool rank_column) {
  make_dirs(dirname_of(path));
  FILE* fp = std::fopen(path.c_str(), "wb");
  if (!fp) HEAT3D_THROW("cannot open '" << path << "' for writing: " << std::strerror(errno));
  std::string head = "TITLE=\"out\"\n";
  head += rank_column ? "VARIABLES = \"X\", \"Y\", \"Z\", \"T\", \"rank\"\n"
                      : "VARIABLES = \"X\", \"Y\", \"Z\", \"T\"\n";
  std::fwrite(head.data(), 1, head.size(), fp);
  for (const Zone& z : zones) {
    const int64_t ei = z.hi[0] - z.lo[0], ej = z.hi[1] - z.lo[1], ek = z.hi[2] - z.lo[2];
    char zh[160];
    int zn = std::snprintf(zh, sizeof(zh), "ZONE T = \"%d\", I=%lld, J=%lld, K=%lld, F=POINT\n", z.title,
                           (long long)ei, (long long)ej, (long long)ek);
    std::fwrite(zh, 1, zn, fp);
    // format one k plane per task, in parallel, then write in order
    const int64_t line_max = rank_column ? 4 * 15 + 5 + 1 : 4 * 15 + 1;
    const int64_t batch = 64;
    for (int64_t kb = 0; kb < ek; kb += batch) {
      const int64_t ke = std::min(ek, kb + batch);
      std::vector<std::string> bufs(ke - kb);
#pragma omp parallel for schedule(dynamic)
      for (int64_t kk = kb; kk < ke; ++kk) {
        std::string& s = bufs[kk - kb];
        s.resize(static_cast<std::size_t>(ei * ej * (line_max + 8)));
        char* o = &s[0];
        const int64_t gk = z.lo[2] + kk;
        const double zc = static_cast<double>(gk) * h[2];
        for (int64_t jj = 0; jj < ej; ++jj) {
          const int64_t gj = z.lo[1] + jj;
          const double yc = static_cast<double>(gj) * h[1];
          for (int64_t ii = 0; ii < ei; ++ii) {
            const int64_t gi = z.lo[0] + ii;
            const double xc = static_cast<double>(gi) * h[0];
            o += fmt_e(o, xc);
            o += fmt_e(o, yc);
            o += fmt_e(o, zc);
            o += fmt_e(o, field[(gi * N[1] + gj) * N[2] + gk]);
            if (rank_column) o += std::snprintf(o, 16, "%5d", z.rank);
            *o++ = '\n';
          }
        }
        s.resize(static_cast<std::size_t>(o - &s[0]));
      }
      for (auto& s : bufs) std::fwrite(s.data(), 1, s.size(), fp);
    }
  }
  if (std::fclose(fp) != 0) HEAT3D_THROW("error closing '" << path << "'");
}

static std::string esc(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += c;
  }
  return o + "\"";
}

void Json::set(const std::string& k, const std::string& v) { kv_.push_back({k, esc(v)}); }
void Json::set(const std::string& k, double v) {
  char b[64];
  std::snprintf(b, sizeof(b), "%.17g", v);
  std::string s = b;
  if (s == "inf" || s == "-inf" || s == "nan" || s == "-nan") s = "null";
  kv_.push_back({k, s});
}
void Json::set(const std::string& k, int64_t v) { kv_.push_back({k, std::to_string(v)}); }
void Json::set_bool(const std::string& k, bool v) { kv_.push_back({k, v ? "true" : "false"}); }
void Json::set_raw(const std::string& k, const std::string& raw) { kv_.push_back({k, raw}); }

std::string Json::dump() const {
  std::string o = "{";
  for (std::size_t i = 0; i < kv_.size(); ++i) {
    if (i) o += ", ";
    o += esc(kv_[i].first) + ": " + kv_[i].second;
  }
  return o + "}";
}

std::map<std::string, std::string> Json::parse_flat(const std::string& t) {
  // Parses {"k": value, ...} where value is a number, string, bool or a
  // flat [..] array (kept as raw text).  Enough for our own meta files.
  std::map<std::string, std::string> m;
  std::size_t i = t.find('{');
  if (i == std::string::npos) HEAT3D_THROW("json: no object");
  ++i;
  auto skip = [&]() {
    while (i < t.size() && (t[i] == ' ' || t[i] == '\n' || t[i] == '\t' || t[i] == '\r' || t[i] == ','))
      ++i;
  };
  auto str = [&]() {
    HEAT3D_CHECK(t[i] == '"', "json: expected string at " << i);
    std::string s;
    ++i;
    while (i < t.size() && t[i] != '"') {
      if (t[i] == '\\') ++i;
      s += t[i++];
    }
    ++i;
    return s;
  };
  while (true) {
    skip();
    if (i >= t.size() || t[i] == '}') break;
    std::string k = str();
    skip();
    HEAT3D_CHECK(t[i] == ':', "json: expected ':'");
    ++i;
    skip();
    std::string v;
    if (t[i] == '"') v = str();
    else if (t[i] == '[') {
      std::size_t e = t.find(']', i);
      v = t.substr(i, e - i + 1);
      i = e + 1;
    } else {
      std::size_t s = i;
      while (i < t.size() && t[i] != ',' && t[i] != '}') ++i;
      v = t.substr(s, i - s);
      while (!v.empty() && (v.back() == ' ' || v.back() == '\n')) v.pop_back();
    }
    m[k] = v;
  }
  return m;
}

std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) HEAT3D_THROW("cannot read '" << path << "'");
  std::ostringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

void write_file_atomic(const std::string& path, const std::string& content) {
  make_dirs(dirname_of(path));
  const std::string tmp = path + ".tmp";
  int fd = open_raw(tmp, true, true);
  pwrite_all(fd, content.data(), content.size(), 0);
  fsync_raw(fd);
  close_raw(fd);
  rename_durable(tmp, path);
}

int open_raw(const std::string& path, bool write, bool truncate) {
  int fd = write ? ::open(path.c_str(), O_WRONLY | O_CREAT | (truncate ? O_TRUNC : 0), 0644)
                 : ::open(path.c_str(), O_RDONLY);
  if (fd < 0) HEAT3D_THROW("open(" << path << ") failed: " << std::strerror(errno));
  return fd;
}

void truncate_raw(int fd, int64_t size) {
  if (::ftruncate(fd, size) != 0) HEAT3D_THROW("ftruncate failed: " << std::strerror(errno));
}

void fsync_raw(int fd) {
  if (::fsync(fd) != 0 && errno != EINVAL) HEAT3D_THROW("fsync failed: " << std::strerror(errno));
}

int64_t file_size(const std::string& path) {
  struct stat st;
  if (::stat(path.c_str(), &st) != 0) return -1;
  return (int64_t)st.st_size;
}

void rename_durable(const std::string& from, const std::string& to) {
  if (std::rename(from.c_str(), to.c_str()) != 0)
    HEAT3D_THROW("rename '" << from << "' -> '" << to << "' failed: " << std::strerror(errno));
  std::string d = dirname_of(to);
  if (d.empty()) d = ".";
  int fd = ::open(d.c_str(), O_RDONLY | O_DIRECTORY);
  if (fd >= 0) {
    (void)::fsync(fd);
    ::close(fd);
  }
}

std::vector<std::string> list_dir(const std::string& dir) {
  std::vector<std::string> out;
  DIR* d = ::opendir(dir.c_str());
  if (!d) return out;
  while (dirent* e = ::readdir(d)) {
    const std::string n = e->d_name;
    if (n != "." && n != "..") out.push_back(n);
  }
  ::closedir(d);
  return out;
}

void remove_file(const std::string& path) { (void)std::remove(path.c_str()); }

void pwrite_all(int fd, const void* p, std::size_t n, int64_t off) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t w = ::pwrite(fd, c, n, off);
    if (w < 0) {
      if (errno == EINTR) continue;
      HEAT3D_THROW("pwrite failed: " << std::strerror(errno));
    }
    c += w;
    n -= w;
    off += w;
  }
}

void pread_all(int fd, void* p, std::size_t n, int64_t off) {
  char* c = static_cast<char*>(p);
  while (n) {
    ssize_t r = ::pread(fd, c, n, off);
    if (r < 0) {
      if (errno == EINTR) continue;
      HEAT3D_THROW("pread failed: " << std::strerror(errno));
    }
    if (r == 0) HEAT3D_THROW("pread: unexpected end of file");
    c += r;
    n -= r;
    off += r;
  }
}

void close_raw(int fd) {
  if (fd >= 0) ::close(fd);
}

}  // namespace io
}  // namespace heat3d
