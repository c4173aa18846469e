// heat3d-mi355x — solver output: field access, gather to the root, Tecplot
// writers (heat3D.cu:1109-1179) and binary checkpoint / restart.
#include "solver.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <sstream>
#include <thread>

#include <unistd.h>

#include "../comm/net.hpp"
#include "../io/io.hpp"

namespace heat3d {
std::vector<double> Solver::local_field(int idx, bool with_ghosts) {
  be_->sync_all();
  auto& l = local_.at(idx);
  Box b;
  for (int a = 0; a < 3; ++a) {
    b.lo[a] = with_ghosts ? -1 : 0;
    b.hi[a] = l.sd.n[a] + (with_ghosts ? 1 : 0);
  }
  const std::size_t bytes = b.volume() * esize_;
  void* dbuf = be_->alloc(bytes);
  be_->pack_box(dt_, l.field[cur()], l.L, b, dbuf, kCompute);
  std::vector<char> h(bytes);
  be_->copy(h.data(), dbuf, bytes, CopyKind::D2H, kCompute);
  be_->sync(kCompute);
  be_->release(dbuf);
  std::vector<double> out(b.volume());
  for (std::size_t i = 0; i < out.size(); ++i)
    out[i] = dt_ == DType::F64 ? reinterpret_cast<double*>(h.data())[i]
                               : (double)reinterpret_cast<float*>(h.data())[i];
  return out;
}

// Host memory a root-side gather may use: half of the physical RAM, unless
// --host-mem-limit-gb says otherwise.
static double host_mem_limit_bytes(const Config& c) {
  if (c.host_mem_limit_gb > 0) return c.host_mem_limit_gb * 1e9;
  const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGE_SIZE);
  return pages > 0 && psz > 0 ? 0.5 * (double)pages * (double)psz : 64e9;
}

// Staging chunk of the streamed I/O paths (device stage + pinned host buffer).
static std::size_t io_stage_bytes(const Config& c) { return (std::size_t)std::max(1, c.io_stage_mb) << 20; }

// Visit the box `g` (global coords) of local subdomain `l` in x chunks of at
// most stage_bytes: pack the chunk on the device, copy it to pinned host
// memory and call fn(x0, nx, host) with nx planes of g.extent(1) x
// g.extent(2) values (z fastest).  Memory stays bounded by one chunk.
template <typename Fn>
static void stream_box_out(Backend& be, DType dt, std::size_t esize, const void* field, const Layout& L,
                           const Subdomain& sd, const Box& g, std::size_t stage_bytes, Fn fn) {
  const int64_t plane = g.extent(1) * g.extent(2);
  if (plane <= 0 || g.extent(0) <= 0) return;
  const int64_t xc = std::max<int64_t>(1, std::min<int64_t>(g.extent(0), (int64_t)stage_bytes / (plane * esize)));
  void* stage = be.alloc(xc * plane * esize);
  void* host = be.alloc_host(xc * plane * esize);
  try {
    for (int64_t x0 = 0; x0 < g.extent(0); x0 += xc) {
      const int64_t nx = std::min(xc, g.extent(0) - x0);
      Box lb = g;
      for (int a = 0; a < 3; ++a) {
        lb.lo[a] -= sd.gstart[a];
        lb.hi[a] -= sd.gstart[a];
      }
      lb.lo[0] += x0;
      lb.hi[0] = lb.lo[0] + nx;
      be.pack_box(dt, field, L, lb, stage, kCompute);
      be.copy(host, stage, nx * plane * esize, CopyKind::D2H, kCompute);
      be.sync(kCompute);
      fn(x0, nx, static_cast<const char*>(host));
    }
  } catch (...) {
    be.release(stage);
    be.release_host(host);
    throw;
  }
  be.release(stage);
  be.release_host(host);
}

bool Solver::gather_global(std::vector<double>* out) {
  be_->sync_all();
  const int P = comm_->size();
  const bool root = is_root();
  const int p = cur();
  const int64_t* N = dec_.N;
  const double need = 8.0 * (double)N[0] * (double)N[1] * (double)N[2];
  const bool ok = need <= host_mem_limit_bytes(cfg_);
  if (!ok) {
    // every rank throws (same test): no rank is left waiting in a send
    HEAT3D_THROW("gathering the " << N[0] << "x" << N[1] << "x" << N[2] << " field on the root needs " << need / 1e9
                                  << " GB of host memory (limit " << host_mem_limit_bytes(cfg_) / 1e9
                                  << " GB, --host-mem-limit-gb); write per-rank Tecplot zones "
                                     "(--tecplot-layout owned) or a checkpoint instead");
  }
  if (root) out->assign((std::size_t)(N[0] * N[1] * N[2]), 0.0);
  int64_t maxvol = 0;
  for (const auto& s : dec_.subs) maxvol = std::max(maxvol, s.extended_global().volume());
  auto scatter = [&](const Box& g, const char* host) {
    const int64_t ey = g.extent(1), ez = g.extent(2);
    for (int64_t i = 0; i < g.extent(0); ++i)
      for (int64_t j = 0; j < ey; ++j) {
        double* dst = out->data() + ((g.lo[0] + i) * N[1] + (g.lo[1] + j)) * N[2] + g.lo[2];
        const int64_t o = (i * ey + j) * ez;
        if (dt_ == DType::F64) std::memcpy(dst, reinterpret_cast<const double*>(host) + o, ez * 8);
        else
          for (int64_t k = 0; k < ez; ++k) dst[k] = reinterpret_cast<const float*>(host)[o + k];
      }
  };
  void* stage = nullptr;
  std::vector<char> host;
  for (int r = 0; r < P; ++r) {
    const Subdomain& s = dec_.subs[r];
    const Box g = s.extended_global();
    const std::size_t bytes = g.volume() * esize_;
    int li = -1;
    for (std::size_t q = 0; q < local_.size(); ++q)
      if (local_[q].sd.rank == r) li = (int)q;
    if (li >= 0 && root) {
      // the root's own blocks: streamed, no full-block stage
      Local& l = local_[li];
      stream_box_out(*be_, dt_, esize_, l.field[p], l.L, l.sd, g, io_stage_bytes(cfg_), [&](int64_t x0, int64_t nx, const char* h) {
        Box c = g;
        c.lo[0] = g.lo[0] + x0;
        c.hi[0] = c.lo[0] + nx;
        scatter(c, h);
      });
      continue;
    }
    if (!stage && (li >= 0 || root)) {
      stage = be_->alloc(maxvol * esize_);
      host.resize(maxvol * esize_);
    }
    if (li >= 0) {
      Local& l = local_[li];
      Box lb = g;
      for (int a = 0; a < 3; ++a) {
        lb.lo[a] -= s.gstart[a];
        lb.hi[a] -= s.gstart[a];
      }
      be_->pack_box(dt_, l.field[p], l.L, lb, stage, kCompute);
      if (comm_->device_buffers()) {
        comm_->send(stage, bytes, 0, *be_, kCompute);
        be_->sync(kCompute);
      } else {
        be_->sync(kCompute);
        comm_->send(stage, bytes, 0, *be_, kCompute);
      }
    } else if (root) {
      comm_->recv(stage, bytes, r, *be_, kCompute);
      be_->copy(host.data(), stage, bytes, CopyKind::D2H, kCompute);
      be_->sync(kCompute);
      scatter(g, host.data());
    }
  }
  be_->sync_all();
  if (stage) be_->release(stage);
  return root;
}

// Tecplot zone header of heat3D.cu:1148 (title = the rank; --compat: "0").
static std::string zone_header(int title, const Box& z) {
  char zh[192];
  const int n = std::snprintf(zh, sizeof(zh), "ZONE T = \"%d\", I=%lld, J=%lld, K=%lld, F=POINT\n", title,
                              (long long)z.extent(0), (long long)z.extent(1), (long long)z.extent(2));
  return std::string(zh, n);
}

void Solver::write_tecplot(const std::string& path, const std::string& layout_req) {
  const int P = comm_->size();
  bool ref_legal = true;
  for (int a = 0; a < 3; ++a) ref_legal &= (dec_.N[a] - 1) % dec_.topo.dims[a] == 0;
  std::string layout = layout_req;
  if (layout == "auto") layout = ref_legal ? "ref" : "owned";
  if (layout == "ref" && !ref_legal)
    HEAT3D_THROW("--tecplot-layout ref needs (N-1) % dims == 0 on every axis (heat3D.cu:375-380)");
  if (layout == "owned" || P == 1) {
    write_tecplot_zones(path);
    return;
  }
  // reference layout: zones share a plane with each neighbour, so a zone
  // holds points of other ranks -> gather on the root (small, reference-legal
  // grids; gather_global refuses grids that exceed host memory)
  std::vector<double> g;
  const bool root = gather_global(&g);
  if (!root) return;
  std::vector<io::Zone> zones;
  for (int r = 0; r < P; ++r) {
    io::Zone z;
    z.rank = r;
    z.title = cfg_.compat ? 0 : r;  // the reference always printed rank 0's id (heat3D.cu:1148)
    // reference chunks: c = (N-1)/dims + 1 points, sharing one plane with
    // each neighbour (heat3D.cu:385-389, 1135)
    auto c = dec_.topo.coords(r);
    for (int a = 0; a < 3; ++a) {
      const int64_t ch = (dec_.N[a] - 1) / dec_.topo.dims[a] + 1;
      z.lo[a] = c[a] * (ch - 1);
      z.hi[a] = z.lo[a] + ch;
    }
    zones.push_back(z);
  }
  io::write_tecplot(path, g, dec_.N, phys_.h, zones, P > 1);
}

// Per-rank parallel Tecplot output (replaces the reference's gather to rank 0
// and serial write, heat3D.cu:1112-1179).  Every line has a fixed width
// ("%15.5e" x 4 [+ "%5d"] + '\n'), so each rank computes the byte offset of
// its zone from the decomposition alone, formats its extended box chunk by
// chunk and pwrite()s it; the root writes the file header.  No process holds
// more than one staging chunk, whatever the grid size.
void Solver::write_tecplot_zones(const std::string& path) {
  be_->sync_all();
  const int P = comm_->size();
  HEAT3D_CHECK(P < 100000, "rank column is %5d");
  const bool rank_column = P > 1;
  const int64_t line = 4 * 15 + (rank_column ? 5 : 0) + 1;
  std::string head = "TITLE=\"out\"\n";
  head += rank_column ? "VARIABLES = \"X\", \"Y\", \"Z\", \"T\", \"rank\"\n" : "VARIABLES = \"X\", \"Y\", \"Z\", \"T\"\n";
  std::vector<int64_t> off(P + 1);
  off[0] = (int64_t)head.size();
  for (int r = 0; r < P; ++r) {
    const Box z = dec_.subs[r].extended_global();
    off[r + 1] = off[r] + (int64_t)zone_header(cfg_.compat ? 0 : r, z).size() + z.volume() * line;
  }
  if (is_root()) {
    io::make_dirs(io::dirname_of(path));
    int fd = io::open_raw(path, true, true);
    io::pwrite_all(fd, head.data(), head.size(), 0);
    io::truncate_raw(fd, off[P]);
    io::close_raw(fd);
  }
  comm_->barrier(*be_);
  const int p = cur();
  int fd = io::open_raw(path, true);
  for (auto& l : local_) {
    const int r = l.sd.rank;
    const Box g = l.sd.extended_global();
    const std::string zh = zone_header(cfg_.compat ? 0 : r, g);
    io::pwrite_all(fd, zh.data(), zh.size(), off[r]);
    const int64_t body = off[r] + (int64_t)zh.size();
    const int64_t ex = g.extent(0), ey = g.extent(1), ez = g.extent(2);
    // the zone runs k outermost, i innermost: stream z chunks of the box
    const int64_t kc = std::max<int64_t>(1, std::min<int64_t>(ez, io_stage_bytes(cfg_) / std::max<int64_t>(1, ex * ey * esize_)));
    void* stage = be_->alloc(ex * ey * kc * esize_);
    std::vector<char> host(ex * ey * kc * esize_);
    std::string text;
    for (int64_t k0 = 0; k0 < ez; k0 += kc) {
      const int64_t nk = std::min(kc, ez - k0);
      Box lb = g;
      for (int a = 0; a < 3; ++a) {
        lb.lo[a] -= l.sd.gstart[a];
        lb.hi[a] -= l.sd.gstart[a];
      }
      lb.lo[2] += k0;
      lb.hi[2] = lb.lo[2] + nk;
      be_->pack_box(dt_, l.field[p], l.L, lb, stage, kCompute);  // x, y, z-chunk order, z fastest
      be_->copy(host.data(), stage, ex * ey * nk * esize_, CopyKind::D2H, kCompute);
      be_->sync(kCompute);
      text.resize((std::size_t)(nk * ey * ex * line));
      // no exception may leave the parallel region (std::terminate): a bad
      // line width is flagged and thrown after it
      int bad_width = 0;
#pragma omp parallel for schedule(static) reduction(max : bad_width)
      for (int64_t kk = 0; kk < nk; ++kk) {
        char buf[128];  // one line: 4 x 15 + 5 + 1 characters
        const double zc = (double)(g.lo[2] + k0 + kk) * phys_.h[2];
        for (int64_t j = 0; j < ey; ++j) {
          const double yc = (double)(g.lo[1] + j) * phys_.h[1];
          char* o = &text[(std::size_t)((kk * ey + j) * ex * line)];
          for (int64_t i = 0; i < ex; ++i) {
            const double xc = (double)(g.lo[0] + i) * phys_.h[0];
            const int64_t idx = (i * ey + j) * nk + kk;
            const double v = dt_ == DType::F64 ? reinterpret_cast<const double*>(host.data())[idx]
                                               : (double)reinterpret_cast<const float*>(host.data())[idx];
            int w = std::snprintf(buf, sizeof(buf), "%15.5e%15.5e%15.5e%15.5e", xc, yc, zc, v);
            if (rank_column) w += std::snprintf(buf + w, sizeof(buf) - w, "%5d", r);
            if (w != line - 1) {
              bad_width = std::max(bad_width, w + 1);
              w = std::min(w, (int)line - 1);
            }
            std::memcpy(o, buf, w);
            o[w] = '\n';
            o += line;
          }
        }
      }
      if (bad_width) {
        io::close_raw(fd);
        HEAT3D_THROW("tecplot: line width " << bad_width - 1 << " != " << line - 1);
      }
      io::pwrite_all(fd, text.data(), text.size(), body + k0 * ey * ex * line);
    }
    be_->release(stage);
  }
  io::close_raw(fd);
  comm_->barrier(*be_);
}

// Order-independent checksum of the global field: Σ bit patterns of every
// value (u64 for fp64, u32 zero-extended for fp32), mod 2^64.
static unsigned long long host_bitsum(const char* p, int64_t n, DType dt) {
  unsigned long long s = 0;
  if (dt == DType::F64) {
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
    for (int64_t i = 0; i < n; ++i) s += q[i];
  } else {
    const unsigned* q = reinterpret_cast<const unsigned*>(p);
    for (int64_t i = 0; i < n; ++i) s += q[i];
  }
  return s;
}

unsigned long long Solver::allreduce_sum_u64(unsigned long long v) {
  if (comm_->all_local() || comm_->size() == 1) return v;
  void* d = be_->alloc(8);
  be_->copy(d, &v, 8, CopyKind::H2D, kReduce);
  comm_->allreduce(d, 1, RedType::U64, RedOp::Sum, *be_, kReduce);
  be_->copy(&v, d, 8, CopyKind::D2H, kReduce);
  be_->sync(kReduce);
  be_->release(d);
  return v;
}

// Checkpoint (new; the reference has no restart), crash-safe:
//   1. every rank pwrite()s its extended box, streamed in bounded chunks, into
//      field.<iter>.raw.tmp (the root creates and sizes it), then fsync()s;
//   2. the root renames it to field.<iter>.raw (complete);
//   3. the root atomically replaces meta.json (tmp + fsync + rename), which
//      names that file with its byte size and checksum;
//   4. older field.*.raw files are removed.
// A crash at any point leaves meta.json naming a complete field file;
// restart checks the file size and the checksum.
void Solver::save_checkpoint(const std::string& dir) {
  be_->sync_all();
  HostState hs = state();
  const int p = cur();
  const int64_t* N = dec_.N;
  const std::string name = "field." + std::to_string(issued_) + ".raw";
  const std::string path = dir + "/" + name, tmp = path + ".tmp";
  const int64_t total = N[0] * N[1] * N[2] * (int64_t)esize_;
  if (is_root()) {
    io::make_dirs(dir);
    int fd = io::open_raw(tmp, true, true);
    io::truncate_raw(fd, total);
    io::close_raw(fd);
  }
  comm_->barrier(*be_);
  unsigned long long sum = 0;
  {
    int fd = io::open_raw(tmp, true);
    for (auto& l : local_) {
      const Box g = l.sd.extended_global();
      const int64_t ey = g.extent(1), ez = g.extent(2);
      stream_box_out(*be_, dt_, esize_, l.field[p], l.L, l.sd, g, io_stage_bytes(cfg_), [&](int64_t x0, int64_t nx, const char* h) {
        sum += host_bitsum(h, nx * ey * ez, dt_);
        // contiguous runs in the file: the whole chunk (x slabs), a plane's
        // rows (y splits), else one row at a time (z splits)
        if (ez == N[2] && ey == N[1]) {
          io::pwrite_all(fd, h, nx * ey * ez * esize_, (g.lo[0] + x0) * N[1] * N[2] * esize_);
          return;
        }
        for (int64_t i = 0; i < nx; ++i) {
          const int64_t gi = g.lo[0] + x0 + i;
          if (ez == N[2]) {
            io::pwrite_all(fd, h + i * ey * ez * esize_, ey * ez * esize_, (gi * N[1] + g.lo[1]) * N[2] * esize_);
            continue;
          }
          for (int64_t j = 0; j < ey; ++j) {
            const int64_t off = ((gi * N[1] + (g.lo[1] + j)) * N[2] + g.lo[2]) * esize_;
            io::pwrite_all(fd, h + (i * ey + j) * ez * esize_, ez * esize_, off);
          }
        }
      });
    }
    io::fsync_raw(fd);
    io::close_raw(fd);
  }
  sum = allreduce_sum_u64(sum);
  comm_->barrier(*be_);
  if (is_root()) {
    io::rename_durable(tmp, path);
    io::Json j;
    j.set("format", std::string("heat3d-checkpoint-v2"));
    j.set("field", name);
    j.set("bytes", total);
    char ck[32];
    std::snprintf(ck, sizeof(ck), "%016llx", sum);
    j.set("checksum", std::string(ck));
    j.set("checksum_kind", std::string("sum of value bit patterns mod 2^64"));
    j.set_raw("N", "[" + std::to_string(N[0]) + ", " + std::to_string(N[1]) + ", " + std::to_string(N[2]) + "]");
    j.set("dtype", std::string(dtype_name(dt_)));
    j.set("iteration", (int64_t)issued_);
    j.set("norm", hs.norm);
    j.set("eps", hs.eps);
    j.set("last_residual", hs.last_residual);
    j.set_raw("dims", "[" + std::to_string(dec_.topo.dims[0]) + ", " + std::to_string(dec_.topo.dims[1]) +
                          ", " + std::to_string(dec_.topo.dims[2]) + "]");
    j.set("layout", std::string("global z-fastest, N0*N1*N2 values"));
    io::write_file_atomic(dir + "/meta.json", j.dump() + "\n");
    // older field files, and the temp files of saves that a crash
    // interrupted (a full-grid field.<iter>.raw.tmp each)
    auto ends_with = [](const std::string& s, const char* suf) {
      const std::size_t n = std::strlen(suf);
      return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
    };
    for (const std::string& old : io::list_dir(dir)) {
      const bool is_field = old.rfind("field.", 0) == 0 && (ends_with(old, ".raw") || ends_with(old, ".raw.tmp"));
      if (is_field && old != name) io::remove_file(dir + "/" + old);
    }
  }
  comm_->barrier(*be_);
}

void Solver::load_checkpoint(const std::string& dir) {
  auto meta = io::Json::parse_flat(io::read_file(dir + "/meta.json"));
  const bool v2 = meta["format"] == "heat3d-checkpoint-v2";
  HEAT3D_CHECK(v2 || meta["format"] == "heat3d-checkpoint-v1", "not a heat3d checkpoint: " << dir);
  const std::string Nexp = "[" + std::to_string(dec_.N[0]) + ", " + std::to_string(dec_.N[1]) + ", " +
                           std::to_string(dec_.N[2]) + "]";
  HEAT3D_CHECK(meta["N"] == Nexp, "checkpoint grid " << meta["N"] << " != run grid " << Nexp);
  HEAT3D_CHECK(meta["dtype"] == dtype_name(dt_), "checkpoint dtype " << meta["dtype"] << " != " << dtype_name(dt_));
  const int64_t it = std::atoll(meta["iteration"].c_str());
  const double norm = std::atof(meta["norm"].c_str());
  const int64_t* N = dec_.N;
  const std::string path = dir + "/" + (v2 ? meta["field"] : std::string("field.raw"));
  const int64_t total = N[0] * N[1] * N[2] * (int64_t)esize_;
  HEAT3D_CHECK(io::file_size(path) == total,
               "checkpoint field " << path << " has " << io::file_size(path) << " bytes, expected " << total);
  if (v2) HEAT3D_CHECK(std::atoll(meta["bytes"].c_str()) == total, "checkpoint meta size mismatch");
  int fd = io::open_raw(path, false);
  unsigned long long sum = 0;
  for (auto& l : local_) {
    // the ghosted block (one layer around the owned box), x chunks
    Box lb;
    for (int a = 0; a < 3; ++a) {
      lb.lo[a] = -1;
      lb.hi[a] = l.sd.n[a] + 1;
    }
    const Box ext = l.sd.extended_global();
    const int64_t ey = lb.extent(1), ez = lb.extent(2), plane = ey * ez;
    const int64_t xc = std::max<int64_t>(1, std::min<int64_t>(lb.extent(0), io_stage_bytes(cfg_) / (plane * esize_)));
    std::vector<char> host(xc * plane * esize_);
    void* stage = be_->alloc(host.size());
    for (int64_t x0 = 0; x0 < lb.extent(0); x0 += xc) {
      const int64_t nx = std::min(xc, lb.extent(0) - x0);
      // reads: whole rows are contiguous runs of the file once the box spans
      // z (one read per plane), and whole planes once it spans y too (one
      // read per chunk); otherwise one read per row
      const int64_t gi0 = l.sd.gstart[0] - 1 + x0, gj0 = l.sd.gstart[1] - 1, gk0 = l.sd.gstart[2] - 1;
      if (ez == N[2] && ey == N[1]) {
        io::pread_all(fd, host.data(), nx * plane * esize_, gi0 * N[1] * N[2] * esize_);
      } else if (ez == N[2]) {
        for (int64_t i = 0; i < nx; ++i)
          io::pread_all(fd, host.data() + i * plane * esize_, plane * esize_,
                        ((gi0 + i) * N[1] + gj0) * N[2] * esize_);
      } else {
        for (int64_t i = 0; i < nx; ++i)
          for (int64_t j = 0; j < ey; ++j)
            io::pread_all(fd, host.data() + (i * ey + j) * ez * esize_, ez * esize_,
                          (((gi0 + i) * N[1] + gj0 + j) * N[2] + gk0) * esize_);
      }
      for (int64_t i = 0; i < nx; ++i)
        for (int64_t j = 0; j < ey; ++j) {
          const int64_t gi = gi0 + i, gj = gj0 + j, gk = gk0;
          char* row = host.data() + (i * ey + j) * ez * esize_;
          // checksum over this rank's extended box only (a partition of the grid)
          if (gi >= ext.lo[0] && gi < ext.hi[0] && gj >= ext.lo[1] && gj < ext.hi[1]) {
            const int64_t k0 = ext.lo[2] - gk, k1 = ext.hi[2] - gk;
            sum += host_bitsum(row + k0 * esize_, k1 - k0, dt_);
          }
        }
      Box cb = lb;
      cb.lo[0] = lb.lo[0] + x0;
      cb.hi[0] = cb.lo[0] + nx;
      be_->copy(stage, host.data(), nx * plane * esize_, CopyKind::H2D, kCompute);
      for (int b = 0; b < nbuf_; ++b) be_->unpack_box(dt_, l.field[b], l.L, cb, stage, kCompute);
      be_->sync(kCompute);
    }
    be_->release(stage);
  }
  io::close_raw(fd);
  if (v2) {
    sum = allreduce_sum_u64(sum);
    char ck[32];
    std::snprintf(ck, sizeof(ck), "%016llx", sum);
    HEAT3D_CHECK(meta["checksum"] == ck, "checkpoint field " << path << " checksum " << ck << " != meta "
                                                             << meta["checksum"] << " (corrupt or partial file)");
  }
  be_->copy(hstate_, dstate_, sizeof(DeviceState), CopyKind::D2H, kCompute);
  be_->sync(kCompute);
  hstate_->iter = it;
  hstate_->norm = norm;
  hstate_->done = 0;
  hstate_->conv_iter = -1;
  for (auto& r : hstate_->residual) r = kResidualInitBits;
  be_->copy(dstate_, hstate_, sizeof(DeviceState), CopyKind::H2D, kCompute);
  be_->sync(kCompute);
  issued_ = it;
  cur_ = 0;
}

}  // namespace heat3d
