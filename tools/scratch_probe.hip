// scratch_probe.hip -- how the ROCm runtime backs private (scratch) segments on this GPU.
//
// Two recorded runs of the engine aborted with HSA_STATUS_ERROR_OUT_OF_RESOURCES while plenty
// of device memory was free.  The runtime backs scratch out of a
// per-agent pool shared by all queues (HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX) and keeps a
// queue's scratch assigned to it when a dispatch needs no more than a threshold
// (HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_CURRENT); bigger needs are "use once".  This probe prints
// both, then measures -- through hipMemGetInfo -- how much a queue retains after dispatches of
// kernels with known private segment sizes (one wave each, and a full grid), and what a
// dispatch costs when its scratch is retained vs use-once.  It never asks for more scratch than
// a few queues' worth, so it cannot exhaust the pool itself.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/scratch_probe tools/scratch_probe.hip -lhsa-runtime64
// run:   GPU_MAX_HW_QUEUES=10 tools/scratch_probe > profiles/rNN_scratch_probe.json
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#define CHECK(x)                                                                             \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                              \
    }                                                                                        \
  } while (0)

// A kernel whose private segment is ~4*DW bytes per lane: a volatile array indexed by lane.
template <int DW>
__global__ void k_scr(uint32_t* out, uint32_t seed) {
  volatile uint32_t buf[DW];
  for (int i = 0; i < DW; ++i) buf[(i * 7 + threadIdx.x) % DW] = seed + i;
  uint32_t acc = 0;
  for (int i = 0; i < DW; i += 97) acc += buf[(i + threadIdx.x) % DW];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

struct Agents {
  std::vector<hsa_agent_t> gpus;
};
static hsa_status_t collect(hsa_agent_t a, void* p) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_GPU)
    static_cast<Agents*>(p)->gpus.push_back(a);
  return HSA_STATUS_SUCCESS;
}

static size_t free_mem() {
  size_t f = 0, t = 0;
  (void)hipMemGetInfo(&f, &t);
  return f;
}

static std::string sysfs_props() {
  // KFD topology of every GPU node: the scratch-related lines
  std::string out;
  for (int n = 0; n < 64; ++n) {
    std::ifstream f("/sys/class/kfd/kfd/topology/nodes/" + std::to_string(n) + "/properties");
    if (!f) continue;
    std::string line, keep;
    bool gpu = false;
    while (std::getline(f, line)) {
      if (line.rfind("simd_count", 0) == 0 && line != "simd_count 0") gpu = true;
      if (line.find("scratch") != std::string::npos || line.find("slots") != std::string::npos ||
          line.find("cu_per_simd") != std::string::npos || line.find("simd_count") != std::string::npos ||
          line.find("max_waves") != std::string::npos || line.find("num_xcc") != std::string::npos)
        keep += (keep.empty() ? "" : "; ") + line;
    }
    if (gpu) out += (out.empty() ? "" : " | ") + std::string("node ") + std::to_string(n) + ": " + keep;
  }
  return out;
}

template <int DW>
static int launch(hipStream_t s, uint32_t* out, int blocks) {
  hipLaunchKernelGGL(k_scr<DW>, dim3(blocks), dim3(64), 0, s, out, 1u);
  CHECK(hipGetLastError());
  CHECK(hipStreamSynchronize(s));
  return 0;
}

// retained bytes on a queue after one dispatch: the drop in free memory
template <int DW>
static long long delta(hipStream_t s, uint32_t* out, int blocks) {
  const size_t f0 = free_mem();
  if (launch<DW>(s, out, blocks)) return -1;
  const size_t f1 = free_mem();
  return (long long)f0 - (long long)f1;
}

template <int DW>
static double us_per_dispatch(hipStream_t s, uint32_t* out, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k_scr<DW>, dim3(1), dim3(64), 0, s, out, 1u);
  (void)hipEventRecord(a, s);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_scr<DW>, dim3(1), dim3(64), 0, s, out, 1u);
  (void)hipEventRecord(b, s);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return 1e3 * ms / reps;
}

int main() {
  CHECK(hipSetDevice(0));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  if (hsa_init() != HSA_STATUS_SUCCESS) return 2;
  Agents ag;
  hsa_iterate_agents(collect, &ag);
  std::printf("{\n  \"device\": \"%s\", \"cus\": %d, \"gpu_max_hw_queues\": \"%s\",\n", prop.gcnArchName,
              prop.multiProcessorCount, std::getenv("GPU_MAX_HW_QUEUES") ? std::getenv("GPU_MAX_HW_QUEUES") : "");
  std::printf("  \"kfd_props\": \"%s\",\n  \"agents\": [", sysfs_props().c_str());
  hsa_agent_t agent{};
  for (size_t i = 0; i < ag.gpus.size(); ++i) {
    uint64_t mx = 0, cur = 0;
    uint32_t cu = 0, wpc = 0, xcc = 0;
    hsa_agent_get_info(ag.gpus[i], (hsa_agent_info_t)HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX, &mx);
    hsa_agent_get_info(ag.gpus[i], (hsa_agent_info_t)HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_CURRENT, &cur);
    hsa_agent_get_info(ag.gpus[i], (hsa_agent_info_t)HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT, &cu);
    hsa_agent_get_info(ag.gpus[i], (hsa_agent_info_t)HSA_AMD_AGENT_INFO_MAX_WAVES_PER_CU, &wpc);
    hsa_agent_get_info(ag.gpus[i], (hsa_agent_info_t)HSA_AMD_AGENT_INFO_NUM_XCC, &xcc);
    std::printf("%s{\"scratch_limit_max\": %llu, \"scratch_limit_current\": %llu, \"cus\": %u, \"max_waves_per_cu\": %u, "
                "\"num_xcc\": %u}",
                i ? ", " : "", (unsigned long long)mx, (unsigned long long)cur, cu, wpc, xcc);
    if (i == 0) agent = ag.gpus[i];
  }
  std::printf("],\n");
  const double slots = 64.0 * 32.0 * prop.multiProcessorCount;  // lanes x wave slots (model)
  uint32_t* out = nullptr;
  CHECK(hipMalloc(&out, sizeof(uint32_t) * 64 * 8192));
  hipStream_t s[6];
  for (auto& x : s) CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  (void)free_mem();
  std::printf("  \"model_bytes_per_lane_byte\": %.0f,\n  \"retained\": [\n", slots);
  struct Row {
    const char* what;
    long long d;
  };
  std::vector<Row> rows;
  rows.push_back({"s0 one wave 1.3K-dword frame (~5.2 KB)", delta<1300>(s[0], out, 1)});
  rows.push_back({"s0 again, same frame", delta<1300>(s[0], out, 1)});
  rows.push_back({"s0 one wave ~2.2 KB frame (smaller)", delta<560>(s[0], out, 1)});
  rows.push_back({"s1 full grid (8192 waves) ~2.2 KB frame", delta<560>(s[1], out, 8192)});
  rows.push_back({"s1 one wave ~5.2 KB frame (grows)", delta<1300>(s[1], out, 1)});
  rows.push_back({"s2 one wave ~9.4 KB frame", delta<2350>(s[2], out, 1)});
  rows.push_back({"s2 one wave ~9.4 KB frame, again", delta<2350>(s[2], out, 1)});
  rows.push_back({"s3 one wave ~4.2 KB frame", delta<1060>(s[3], out, 1)});
  for (size_t i = 0; i < rows.size(); ++i)
    std::printf("    {\"step\": \"%s\", \"free_mem_drop_bytes\": %lld, \"drop_per_model_slot\": %.1f}%s\n", rows[i].what,
                rows[i].d, rows[i].d / slots, i + 1 < rows.size() ? "," : "");
  std::printf("  ],\n");
  const double t_ret = us_per_dispatch<1300>(s[0], out, 200);
  const double t_big = us_per_dispatch<2350>(s[2], out, 200);
  const double t_none = us_per_dispatch<1>(s[4], out, 200);
  std::printf("  \"us_per_1wave_dispatch\": {\"no_scratch\": %.2f, \"frame_5k_retained_queue\": %.2f, \"frame_9k\": %.2f}",
              t_none, t_ret, t_big);
  // the same dispatches with the runtime's retain threshold lowered below them (every scratch
  // dispatch use-once), then restored
  uint64_t cur = 0;
  hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_CURRENT, &cur);
  const size_t f0 = free_mem();
  const hsa_status_t st = hsa_amd_agent_set_async_scratch_limit(agent, 1u << 20);
  const size_t f1 = free_mem();
  double t_once = -1, t_once_big = -1;
  long long d_once = 0;
  if (st == HSA_STATUS_SUCCESS) {
    t_once = us_per_dispatch<1300>(s[0], out, 200);
    t_once_big = us_per_dispatch<2350>(s[2], out, 200);
    d_once = delta<1300>(s[5], out, 1);
    (void)hsa_amd_agent_set_async_scratch_limit(agent, cur);
  }
  std::printf(",\n  \"use_once\": {\"set_limit_status\": %d, \"freed_by_lowering_bytes\": %lld, "
              "\"us_per_1wave_dispatch_5k\": %.2f, \"us_per_1wave_dispatch_9k\": %.2f, \"retained_after_one_wave\": %lld}\n}\n",
              (int)st, (long long)f1 - (long long)f0, t_once, t_once_big, d_once);
  for (auto& x : s) (void)hipStreamDestroy(x);
  (void)hipFree(out);
  return 0;
}
