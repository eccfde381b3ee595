// lora_aql.hip — allocation-free synchronous dispatch for the C++ drop-in (host code only).
//
// The reference's lora_demodulate performs no heap allocation once its workspace exists
// (no_alloc_test.cpp:90-99 counts every global operator new during the call).  Every HIP
// runtime call that enqueues work - a kernel launch, an async copy, a stream
// synchronisation - allocates a command object with operator new (measured per call by
// tests/native/alloc_probe.cpp: 3 launches + 3 copies/syncs = 8 allocations per frame).
// So the drop-in's per-frame path does not go through the HIP runtime at all:
//
//   * lora_demod_batch runs with a LaunchRecord installed (lora_internal.h): the same host
//     logic picks the same kernels, grids and arguments, which are recorded, not launched;
//   * the frame's samples and outputs live in pinned host memory the kernels read and
//     write directly (one small frame: the PCIe round trips cost less than two copies);
//   * this file writes the recorded launches as AQL kernel-dispatch packets into a queue
//     of its own on the device's HSA agent, rings the doorbell and spins on the last
//     packet's completion signal.  Packets, kernel arguments and the signal are memory
//     set up once in aql_create; kernel objects are looked up once per kernel.
//
// Kernel objects: aql_create loads this library's own gfx950 code objects (the clang
// offload bundles in its .hip_fatbin section, read from the file dladdr names) into HSA
// executables on the device's agent; a kernel's symbol is found by the device name
// hipKernelNameRefByPtr gives for its host stub.  The HIP runtime keeps its own copy for
// every other call.
#include <dlfcn.h>
#include <elf.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <mutex>
#include <vector>

#include "lora_internal.h"

namespace lora {

namespace {

constexpr unsigned kSlotBytes = 1024;  // kernarg slot per packet (explicit + 256 hidden)
constexpr int kCache = 256;  // kernel objects resolved (the drop-in's warm-up: every SF and window)
constexpr int kMaxExec = 8;

struct AqlKernel {
  const void* fn;
  uint64_t object;
  uint32_t kernarg, group, priv;
};

}  // namespace

struct AqlQueue {
  hsa_agent_t agent{};
  hsa_queue_t* q = nullptr;
  hsa_signal_t done{};
  unsigned char* kernarg = nullptr;
  hsa_executable_t exec[kMaxExec]{};
  int nexec = 0;
  AqlKernel k[kCache];
  int nk = 0;
  bool hsa_up = false;
  bool broken = false;  // a call timed out with work in flight (aql_run refuses, -63)
  // LORA_MI355X_AQL_PROFILE=1 at aql_create: one completion signal per packet and the
  // queue's dispatch timestamps, read back after every call (lora_aql_last_profile)
  bool prof = false;
  hsa_signal_t psig[LaunchRecord::kMax]{};
};

namespace {

struct AgentFind {
  uint32_t bdf;
  uint32_t domain;
  hsa_agent_t gpu{};
  bool found = false;
};

hsa_status_t find_gpu(hsa_agent_t a, void* data) {
  AgentFind* f = static_cast<AgentFind*>(data);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0, dom = 0;
  hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
  hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
  if (bdf == f->bdf && dom == f->domain) {
    f->gpu = a;
    f->found = true;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// the system (host) pool kernel arguments are allocated from
struct PoolFind {
  hsa_amd_memory_pool_t pool{};
  bool found = false;
};

hsa_status_t find_kernarg_pool(hsa_amd_memory_pool_t p, void* data) {
  PoolFind* f = static_cast<PoolFind*>(data);
  hsa_amd_segment_t seg;
  if (hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) {
    f->pool = p;
    f->found = true;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t find_cpu_pool(hsa_agent_t a, void* data) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_CPU)
    return HSA_STATUS_SUCCESS;
  hsa_amd_agent_iterate_memory_pools(a, find_kernarg_pool, data);
  return static_cast<PoolFind*>(data)->found ? HSA_STATUS_INFO_BREAK : HSA_STATUS_SUCCESS;
}

const AqlKernel* kernel_of(AqlQueue* Q, const void* fn) {
  for (int i = 0; i < Q->nk; ++i)
    if (Q->k[i].fn == fn) return &Q->k[i];
  if (Q->nk == kCache) return nullptr;
  // first use of this kernel: its device name, then the symbol in one of the executables
  const char* name = hipKernelNameRefByPtr(fn, nullptr);
  if (!name) return nullptr;
  char buf[512];
  const size_t len = std::strlen(name);
  if (len + 4 > sizeof(buf)) return nullptr;
  std::memcpy(buf, name, len);
  std::memcpy(buf + len, ".kd", 4);
  hsa_executable_symbol_t sym{};
  bool found = false;
  for (int e = 0; e < Q->nexec && !found; ++e)
    for (const char* nm : {name, (const char*)buf}) {  // the kernel, or its descriptor's name
      hsa_agent_t ag = Q->agent;
      hsa_symbol_kind_t kind;
      if (hsa_executable_get_symbol_by_name(Q->exec[e], nm, &ag, &sym) == HSA_STATUS_SUCCESS &&
          hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind) == HSA_STATUS_SUCCESS &&
          kind == HSA_SYMBOL_KIND_KERNEL) {
        found = true;
        break;
      }
    }
  if (!found) return nullptr;
  AqlKernel k{fn, 0, 0, 0, 0};
  if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object) !=
          HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kernarg) !=
          HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group) !=
          HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.priv) !=
          HSA_STATUS_SUCCESS)
    return nullptr;
  Q->k[Q->nk] = k;
  return &Q->k[Q->nk++];
}

// The gfx950 code objects of the clang offload bundles in this library's .hip_fatbin
// section (uncompressed bundles: "__CLANG_OFFLOAD_BUNDLE__", an entry count, then per
// entry offset, size, triple length and triple).
bool own_code_objects(std::vector<unsigned char>& file, std::vector<std::pair<size_t, size_t>>& objs,
                      bool& compressed) {
  compressed = false;
  Dl_info info{};
  if (!dladdr(reinterpret_cast<void*>(&aql_create), &info) || !info.dli_fname) return false;
  FILE* fp = std::fopen(info.dli_fname, "rb");
  if (!fp) return false;
  std::fseek(fp, 0, SEEK_END);
  const long n = std::ftell(fp);
  std::fseek(fp, 0, SEEK_SET);
  file.resize(n > 0 ? (size_t)n : 0);
  const bool ok = n > 0 && std::fread(file.data(), 1, file.size(), fp) == file.size();
  std::fclose(fp);
  if (!ok || file.size() < sizeof(Elf64_Ehdr)) return false;
  const Elf64_Ehdr* eh = reinterpret_cast<const Elf64_Ehdr*>(file.data());
  if (std::memcmp(eh->e_ident, ELFMAG, SELFMAG) != 0 || eh->e_shoff == 0 ||
      eh->e_shoff + (size_t)eh->e_shnum * sizeof(Elf64_Shdr) > file.size() || eh->e_shstrndx >= eh->e_shnum)
    return false;
  const Elf64_Shdr* sh = reinterpret_cast<const Elf64_Shdr*>(file.data() + eh->e_shoff);
  const Elf64_Shdr& strs = sh[eh->e_shstrndx];
  for (int i = 0; i < eh->e_shnum; ++i) {
    if (sh[i].sh_name >= strs.sh_size) continue;
    const char* nm = reinterpret_cast<const char*>(file.data() + strs.sh_offset + sh[i].sh_name);
    if (std::strcmp(nm, ".hip_fatbin") != 0 || sh[i].sh_offset + sh[i].sh_size > file.size()) continue;
    static const char kMagic[] = "__CLANG_OFFLOAD_BUNDLE__";
    const size_t lo = sh[i].sh_offset, hi = lo + sh[i].sh_size;
    for (size_t pos = lo; pos + 32 <= hi; pos += 8) {  // bundles start 8-byte aligned
      // a compressed bundle ("CCOB", --offload-compress) is not parsed: aql_create reports it
      if (std::memcmp(file.data() + pos, "CCOB", 4) == 0) compressed = true;
      if (std::memcmp(file.data() + pos, kMagic, 24) != 0) continue;
      uint64_t cnt;
      std::memcpy(&cnt, file.data() + pos + 24, 8);
      size_t p = pos + 32;
      for (uint64_t e = 0; e < cnt && p + 24 <= hi; ++e) {
        uint64_t off, size, tlen;
        std::memcpy(&off, file.data() + p, 8);
        std::memcpy(&size, file.data() + p + 8, 8);
        std::memcpy(&tlen, file.data() + p + 16, 8);
        if (p + 24 + tlen > hi) break;
        const std::string triple(reinterpret_cast<const char*>(file.data() + p + 24), tlen);
        p += 24 + tlen;
        if (triple.find("gfx950") != std::string::npos && pos + off + size <= hi)
          objs.emplace_back(pos + off, (size_t)size);
      }
    }
  }
  return !objs.empty();
}

double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

// The last profiled aql_run (any queue, any thread; diagnostics only): packets, the
// system-domain timestamps of the doorbell, each packet's start/end and the host's
// observation of the completion.
struct LastProfile {
  std::mutex mu;
  AqlQueue* q = nullptr;
  int n = 0;
  uint64_t bell = 0, seen = 0;
};
LastProfile& last_profile() {
  static LastProfile p;
  return p;
}

uint64_t sys_ts() {
  uint64_t t = 0;
  hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &t);
  return t;
}

}  // namespace

int aql_create(int device, AqlQueue** out) {
  *out = nullptr;
  int bus = 0, dev = 0, dom = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess)
    return -101;
  AqlQueue* Q = new AqlQueue();
  if (hsa_init() != HSA_STATUS_SUCCESS) {
    delete Q;
    return -102;
  }
  Q->hsa_up = true;
  int rc = 0;
  do {
    // HSA_AMD_AGENT_INFO_BDFID: bus << 8 | device << 3 | function
    AgentFind af{(uint32_t)(((bus & 0xff) << 8) | ((dev & 0x1f) << 3)), (uint32_t)dom};
    hsa_iterate_agents(find_gpu, &af);
    if (!af.found) {
      rc = -105;
      break;
    }
    Q->agent = af.gpu;
    PoolFind pf;
    hsa_iterate_agents(find_cpu_pool, &pf);
    if (!pf.found) {
      rc = -106;
      break;
    }
    void* ka = nullptr;
    if (hsa_amd_memory_pool_allocate(pf.pool, (size_t)LaunchRecord::kMax * kSlotBytes, 0, &ka) !=
        HSA_STATUS_SUCCESS) {
      rc = -107;
      break;
    }
    Q->kernarg = static_cast<unsigned char*>(ka);
    if (hsa_amd_agents_allow_access(1, &Q->agent, nullptr, ka) != HSA_STATUS_SUCCESS) {
      rc = -108;
      break;
    }
    uint32_t qmin = 0;
    hsa_agent_get_info(Q->agent, HSA_AGENT_INFO_QUEUE_MIN_SIZE, &qmin);
    const uint32_t qsize = qmin > 64 ? qmin : 64;
    if (hsa_queue_create(Q->agent, qsize, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &Q->q) !=
        HSA_STATUS_SUCCESS) {
      Q->q = nullptr;
      rc = -109;
      break;
    }
    if (hsa_signal_create(0, 0, nullptr, &Q->done) != HSA_STATUS_SUCCESS) {
      Q->done.handle = 0;
      rc = -110;
      break;
    }
    const char* pe = std::getenv("LORA_MI355X_AQL_PROFILE");
    if (pe && pe[0] == '1' && hsa_amd_profiling_set_profiler_enabled(Q->q, 1) == HSA_STATUS_SUCCESS) {
      Q->prof = true;
      for (hsa_signal_t& sg : Q->psig)
        if (hsa_signal_create(0, 0, nullptr, &sg) != HSA_STATUS_SUCCESS) {
          sg.handle = 0;
          Q->prof = false;
        }
    }
    // this library's gfx950 code objects, loaded for the agent
    std::vector<unsigned char> file;
    std::vector<std::pair<size_t, size_t>> objs;
    bool compressed = false;
    if (!own_code_objects(file, objs, compressed) || objs.size() > (size_t)kMaxExec) {
      rc = objs.empty() && compressed ? -111 : -103;  // -111: built with --offload-compress
      break;
    }
    for (const auto& o : objs) {
      hsa_code_object_reader_t rd{};
      hsa_executable_t ex{};
      if (hsa_code_object_reader_create_from_memory(file.data() + o.first, o.second, &rd) != HSA_STATUS_SUCCESS) {
        rc = -104;
        break;
      }
      if (hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &ex) !=
          HSA_STATUS_SUCCESS) {
        hsa_code_object_reader_destroy(rd);
        rc = -104;
        break;
      }
      Q->exec[Q->nexec++] = ex;
      const bool loaded = hsa_executable_load_agent_code_object(ex, Q->agent, rd, nullptr, nullptr) ==
                              HSA_STATUS_SUCCESS &&
                          hsa_executable_freeze(ex, nullptr) == HSA_STATUS_SUCCESS;
      hsa_code_object_reader_destroy(rd);  // loaded code does not depend on the reader
      if (!loaded) {
        rc = -104;
        break;
      }
    }
  } while (false);
  if (rc != 0) {
    aql_destroy(Q);
    return rc;
  }
  *out = Q;
  return 0;
}

void aql_destroy(AqlQueue* Q) {
  if (!Q) return;
  // a queue whose kernels may still be running is left as it is (leaked): destroying it would
  // free the kernarg slots and the signal under them
  if (Q->broken) return;
  {
    LastProfile& P = last_profile();
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.q == Q) P.q = nullptr;
  }
  if (Q->done.handle) hsa_signal_destroy(Q->done);
  for (hsa_signal_t& sg : Q->psig)
    if (sg.handle) hsa_signal_destroy(sg);
  if (Q->q) hsa_queue_destroy(Q->q);
  if (Q->kernarg) hsa_amd_memory_pool_free(Q->kernarg);
  for (int e = 0; e < Q->nexec; ++e) hsa_executable_destroy(Q->exec[e]);
  if (Q->hsa_up) hsa_shut_down();
  delete Q;
}

int aql_run(AqlQueue* Q, const LaunchRecord& r) {
  if (!Q || r.bad || r.n <= 0 || r.n > LaunchRecord::kMax) return -22;
  const AqlKernel* ks[LaunchRecord::kMax];
  for (int i = 0; i < r.n; ++i) {
    ks[i] = kernel_of(Q, r.l[i].fn);
    if (!ks[i]) return -120;
    // Kernel arguments: the explicit ones at the offsets the record packed them at, then
    // - only for kernels that use any - code object v5's implicit block at the next
    // 8-byte boundary (block counts, group sizes, remainders, global offsets, grid dims,
    // dynamic LDS size:
    // the only hidden arguments these kernels' metadata lists, tests/test_aql_kernargs.py).
    const uint32_t ex = r.l[i].arg_bytes, h = (ex + 7u) & ~7u;
    if (ks[i]->kernarg != ex && ks[i]->kernarg != h + 256u) return -121;
    if (ks[i]->kernarg > kSlotBytes || (uint64_t)r.l[i].grid * r.l[i].block > 0xffffffffull) return -22;
  }
  hsa_queue_t* q = Q->q;
  // Every call waits for its last packet's completion, so no earlier kernel still runs
  // (the packet processor may advance the read index a little later: only the ring's space
  // is waited for below) - unless an earlier call timed out: then its kernarg slots, staging
  // and completion signal may still be in use, so refuse before writing anything (-63;
  // callers treat the queue as broken after a -62 and stop using it).
  if (Q->broken) return -63;
  const uint64_t n = (uint64_t)r.n;
  const uint64_t base = hsa_queue_add_write_index_relaxed(q, n);
  while (base + n - hsa_queue_load_read_index_scacquire(q) > q->size) {
  }
  hsa_signal_store_relaxed(Q->done, 1);
  if (Q->prof)
    for (int i = 0; i + 1 < r.n; ++i) hsa_signal_store_relaxed(Q->psig[i], 1);
  hsa_kernel_dispatch_packet_t* ring = static_cast<hsa_kernel_dispatch_packet_t*>(q->base_address);
  for (int i = 0; i < r.n; ++i) {
    const RecordedLaunch& L = r.l[i];
    unsigned char* ka = Q->kernarg + (size_t)i * kSlotBytes;
    const uint32_t ex = L.arg_bytes, h = (ex + 7u) & ~7u;
    std::memcpy(ka, L.args, ex);
    if (ks[i]->kernarg > ex) {
      std::memset(ka + ex, 0, ks[i]->kernarg - ex);
      const uint32_t bc[3] = {L.grid, 1, 1};
      const uint16_t gs[3] = {(uint16_t)L.block, 1, 1};
      const uint16_t grid_dims = 1;
      std::memcpy(ka + h, bc, sizeof(bc));             // hidden_block_count_{x,y,z}
      std::memcpy(ka + h + 12, gs, sizeof(gs));        // hidden_group_size_{x,y,z}
      std::memcpy(ka + h + 64, &grid_dims, 2);         // hidden_grid_dims (remainders, offsets 0)
      std::memcpy(ka + h + 120, &L.lds, 4);            // hidden_dynamic_lds_size
    }
    hsa_kernel_dispatch_packet_t* p = ring + ((base + (uint64_t)i) & (q->size - 1));
    p->workgroup_size_x = (uint16_t)L.block;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->reserved0 = 0;
    p->grid_size_x = L.grid * L.block;
    p->grid_size_y = 1;
    p->grid_size_z = 1;
    p->private_segment_size = ks[i]->priv;
    p->group_segment_size = ks[i]->group + L.lds;
    p->kernel_object = ks[i]->object;
    p->kernarg_address = ka;
    p->reserved2 = 0;
    p->completion_signal = i + 1 == r.n ? Q->done : (Q->prof ? Q->psig[i] : hsa_signal_t{0});
    // in order (barrier bit); system-scope acquire on the first packet (the host wrote the
    // samples) and release on the last (the host reads the outputs), agent scope between
    const uint16_t header =
        (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                   ((i == 0 ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_AGENT) << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                   ((i + 1 == r.n ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_AGENT)
                    << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    __atomic_store_n(reinterpret_cast<uint32_t*>(p), (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
  }
  const uint64_t bell = Q->prof ? sys_ts() : 0;
  hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)(base + n - 1));
  // spin on the completion signal (the call is synchronous, like the reference's); give up
  // after 60 s rather than hang the caller
  const double t0 = now_s();
  while (hsa_signal_wait_scacquire(Q->done, HSA_SIGNAL_CONDITION_LT, 1, 1000000, HSA_WAIT_STATE_ACTIVE) >= 1) {
    if (now_s() - t0 > 60.0) {
      Q->broken = true;  // packets may still run: nothing of this queue may be reused
      return -62;
    }
  }
  if (Q->prof) {
    // the packets' timestamps are read by lora_aql_last_profile, outside the caller's call
    const uint64_t seen = sys_ts();
    LastProfile& P = last_profile();
    std::lock_guard<std::mutex> lk(P.mu);
    P.q = Q;
    P.n = r.n;
    P.bell = bell;
    P.seen = seen;
  }
  return 0;
}

}  // namespace lora

// Diagnostics (include/lora_mi355x.h): the last profiled aql_run as microseconds relative
// to its doorbell - out[0] = packets n, then per packet (start, end), then the host's
// observation of the last completion.  Returns the doubles written (0: nothing profiled).
extern "C" int lora_aql_last_profile(double* out, int cap) {
  lora::LastProfile& P = lora::last_profile();
  std::lock_guard<std::mutex> lk(P.mu);
  if (!out || !P.q || P.n <= 0 || cap < 2 * P.n + 2) return 0;
  uint64_t freq = 0;
  if (hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &freq) != HSA_STATUS_SUCCESS || freq == 0) return 0;
  const double us = 1e6 / (double)freq;
  auto rel = [&](uint64_t t) { return ((double)t - (double)P.bell) * us; };
  for (int i = 0; i < P.n; ++i) {
    hsa_amd_profiling_dispatch_time_t t{};  // system-domain ticks
    if (hsa_amd_profiling_get_dispatch_time(P.q->agent, i + 1 == P.n ? P.q->done : P.q->psig[i], &t) !=
        HSA_STATUS_SUCCESS)
      return 0;
    out[1 + 2 * i] = rel(t.start);
    out[2 + 2 * i] = rel(t.end);
  }
  out[0] = P.n;
  out[1 + 2 * P.n] = rel(P.seen);
  P.q = nullptr;  // read once: the next call reuses the signals
  return 2 * P.n + 2;
}
