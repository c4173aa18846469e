// heat3d-mi355x — CPU backend (OpenMP host kernels, synchronous execution).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <unistd.h>

#include "backend.hpp"

namespace heat3d {

namespace {

struct CpuEvent {
  std::chrono::steady_clock::time_point t;
};

class CpuBackend final : public Backend {
 public:
  explicit CpuBackend(int threads) { cpu::set_threads(threads); }
  const char* name() const override { return "cpu"; }
  bool is_gpu() const override { return false; }

  void* alloc(std::size_t bytes) override {
    void* p = nullptr;
    if (posix_memalign(&p, 256, bytes ? bytes : 256)) HEAT3D_THROW("host allocation of " << bytes << " bytes failed");
    return p;
  }
  void release(void* p) override { std::free(p); }
  bool mem_info(std::size_t* free, std::size_t* total) override {
    // MemAvailable (free + reclaimable page cache), not MemFree
    const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGE_SIZE);
    if (pages <= 0 || psz <= 0) return false;
    *total = (std::size_t)pages * (std::size_t)psz;
    std::FILE* fp = std::fopen("/proc/meminfo", "r");
    if (!fp) return false;
    char line[256];
    bool found = false;
    unsigned long long kb = 0;
    while (!found && std::fgets(line, sizeof(line), fp)) found = std::sscanf(line, "MemAvailable: %llu kB", &kb) == 1;
    std::fclose(fp);
    *free = (std::size_t)kb * 1024;
    return found;
  }
  void* alloc_host(std::size_t bytes) override { return alloc(bytes); }
  void release_host(void* p) override { std::free(p); }
  void copy(void* dst, const void* src, std::size_t bytes, CopyKind, StreamId) override {
    if (bytes) std::memmove(dst, src, bytes);
  }
  void memset(void* dst, int v, std::size_t bytes, StreamId) override { std::memset(dst, v, bytes); }

  void* stream(StreamId) override { return nullptr; }
  Event event_create() override { return new CpuEvent(); }
  void event_destroy(Event e) override { delete static_cast<CpuEvent*>(e); }
  void record(Event e, StreamId) override { static_cast<CpuEvent*>(e)->t = std::chrono::steady_clock::now(); }
  void wait(StreamId, Event) override {}
  bool query(Event) override { return true; }
  void event_sync(Event) override {}
  float elapsed_ms(Event a, Event b) override {
    auto d = static_cast<CpuEvent*>(b)->t - static_cast<CpuEvent*>(a)->t;
    return std::chrono::duration<float, std::milli>(d).count();
  }
  void sync(StreamId) override {}
  void sync_all() override {}

  void init_field(DType t, const InitParams& p, StreamId) override { cpu::init_field(t, p); }
  void stencil(DType t, const StencilParams& p, const KernelSpec&, StreamId) override {
    cpu::stencil(t, p);
  }
  // Reference semantics of the K-step kernels: K single steps through two
  // scratch fields (same ghosts).  Step s updates the box widened by K-1-s
  // planes into [ux0, ux1) and accumulates into residual slot `slot + s`.
  void sweep(DType t, const StencilParams& p, const KernelSpec& k, StreamId) override {
    if (p.state && p.state->done) return;
    const int K = k.K;
    for (int i = 0; i < 2; ++i)
      if (scratch_bytes_[i] < p.L.bytes()) {
        release(scratch_[i]);
        scratch_[i] = alloc(p.L.bytes());
        scratch_bytes_[i] = p.L.bytes();
      }
    cpu::stencil_multi(t, p, K, scratch_[0], scratch_[1]);
  }
  ~CpuBackend() override {
    release(scratch_[0]);
    release(scratch_[1]);
  }
  void pack_box(DType t, const void* f, const Layout& L, const Box& b, void* buf, StreamId) override {
    cpu::pack_box(t, f, L, b, buf);
  }
  void unpack_box(DType t, void* f, const Layout& L, const Box& b, const void* buf, StreamId) override {
    cpu::unpack_box(t, f, L, b, buf);
  }
  void copy_box(DType t, const void* src, const Layout& Ls, const Box& bs, void* dst,
                const Layout& Ld, const Box& bd, StreamId) override {
    cpu::copy_box(t, src, Ls, bs, dst, Ld, bd);
  }
  void check_convergence(DeviceState* st, int slot, StreamId, int count, bool last_only) override {
    HEAT3D_CHECK(!last_only, "cpu backend: no last-residual sweeps");
    for (int i = 0; i < count; ++i) cpu::check_convergence(st, slot + i);
  }
  void error_accumulate(DType t, const void* f, const Layout& L, const Box& box,
                        const int64_t gstart[3], double hy, DeviceState* st, StreamId) override {
    cpu::error_accumulate(t, f, L, box, gstart, hy, st);
  }
  void poke(DType t, void* f, const Layout& L, int64_t i, int64_t j, int64_t k, double value,
            StreamId) override {
    cpu::poke(t, f, L, i, j, k, value);
  }

 private:
  void* scratch_[2] = {nullptr, nullptr};
  std::size_t scratch_bytes_[2] = {0, 0};

 public:
  void box_bitsum(DType t, const void* f, const Layout& L, const Box& b, unsigned long long* out,
                  StreamId) override {
    *out = cpu::box_bitsum(t, f, L, b);
  }
};

}  // namespace

std::unique_ptr<Backend> make_cpu_backend(int threads) {
  return std::unique_ptr<Backend>(new CpuBackend(threads));
}

}  // namespace heat3d
