// Launch-cost microbenchmark for the small-run question: what a chain of
// small dependent launches costs per batch through a stream, a replayed hipGraph, and a hipGraph
// whose kernel nodes get new arguments before every replay.
//   hipcc --offload-arch=gfx950 -O2 -o scripts/launch_bench scripts/launch_bench.hip
//   ./scripts/launch_bench [kernels=25] [blocks=16] [iters=2000]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

struct Args { unsigned* buf; unsigned n; unsigned salt; };

__global__ void k_small(Args a) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.n) a.buf[i] = a.buf[i] * 3u + a.salt;
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 25;
  const int B = argc > 2 ? std::atoi(argv[2]) : 16;
  const int N = argc > 3 ? std::atoi(argv[3]) : 2000;
  const unsigned n = (unsigned)B * 256u;
  unsigned* d; CK(hipMalloc(&d, n * 4));
  CK(hipMemset(d, 0, n * 4));
  char* hin; char* din; unsigned* hout;
  const size_t inb = 64 << 10;
  CK(hipHostMalloc((void**)&hin, inb, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&hout, 64, hipHostMallocDefault));
  CK(hipMalloc(&din, inb));
  hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  using clk = std::chrono::steady_clock;
  auto one = [&](unsigned salt) {
    CK(hipMemcpyAsync(din, hin, inb, hipMemcpyHostToDevice, st));
    for (int k = 0; k < K; ++k) {
      Args a{d, n, salt + (unsigned)k};
      hipLaunchKernelGGL(k_small, dim3(B), dim3(256), 0, st, a);
    }
    CK(hipMemcpyAsync(hout, d, 64, hipMemcpyDeviceToHost, st));
  };
  for (int i = 0; i < 100; ++i) { one(i); CK(hipStreamSynchronize(st)); }
  auto t0 = clk::now();
  for (int i = 0; i < N; ++i) { one(i); CK(hipStreamSynchronize(st)); }
  const double us_stream = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / N;
  // enqueue cost alone (no sync per iteration)
  t0 = clk::now();
  for (int i = 0; i < N; ++i) one(i);
  const double us_enqueue = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / N;
  CK(hipStreamSynchronize(st));

  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  one(0);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  size_t nn = 0; CK(hipGraphGetNodes(g, nullptr, &nn));
  std::vector<hipGraphNode_t> nodes(nn); CK(hipGraphGetNodes(g, nodes.data(), &nn));
  std::vector<hipGraphNode_t> kn;
  for (auto x : nodes) { hipGraphNodeType t; CK(hipGraphNodeGetType(x, &t)); if (t == hipGraphNodeTypeKernel) kn.push_back(x); }
  for (int i = 0; i < 100; ++i) { CK(hipGraphLaunch(ge, st)); CK(hipStreamSynchronize(st)); }
  t0 = clk::now();
  for (int i = 0; i < N; ++i) { CK(hipGraphLaunch(ge, st)); CK(hipStreamSynchronize(st)); }
  const double us_graph = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / N;
  // replay with new arguments (and grid) on every kernel node
  std::vector<Args> av(kn.size());
  t0 = clk::now();
  for (int i = 0; i < N; ++i) {
    for (size_t k = 0; k < kn.size(); ++k) {
      av[k] = Args{d, n, (unsigned)(i + k)};
      void* kp[1] = {&av[k]};
      hipKernelNodeParams p{};
      p.func = (void*)k_small; p.gridDim = dim3(B); p.blockDim = dim3(256); p.sharedMemBytes = 0;
      p.kernelParams = kp; p.extra = nullptr;
      CK(hipGraphExecKernelNodeSetParams(ge, kn[k], &p));
    }
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
  }
  const double us_graph_upd = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / N;
  std::printf("{\"kernels\": %d, \"blocks\": %d, \"kernel_nodes\": %zu, \"us_per_batch_stream\": %.2f, "
              "\"us_enqueue_only\": %.2f, \"us_per_batch_graph\": %.2f, \"us_per_batch_graph_updated\": %.2f}\n",
              K, B, kn.size(), us_stream, us_enqueue, us_graph, us_graph_upd);
  return 0;
}
