// stereo_bench_dp: native C++ data-parallel stereo benchmark over RCCL (no Python in the loop).
//
//   stereo_bench_dp --nproc 8 --model raftstereo-sceneflow --batch 8 --steps 10 --warmup 3
//
// One process per GPU.  With --nproc N the launcher forks N ranks BEFORE any HIP call (no exec) and
// sets RANK / LOCAL_RANK / WORLD_SIZE for each; without it the process reads a torchrun-style env.
// Each rank: engine (batch = per-rank shard, synthetic u8 pairs in pinned host memory, seeded random-init weights),
// then bench.py's step: per-step H2D on the copy stream, sa::dist::DataParallelRunner (frame graph with the point
// clouds reprojected in it + all-gather of disparity on a comm stream, overlapped with the next step).  K steps are timed between barriers; rank 0 prints one JSON line
// with the whole-job FPS (max time over ranks).  The reference has no multi-GPU path.
#include <signal.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "sa/dist.h"
#include "sa/engine.h"
#include "sa/runtime.h"

namespace {
std::string read_file(const std::string& path) {
  if (path.empty()) return std::string();
  std::ifstream f(path, std::ios::binary);
  return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

uint32_t fnv32(const std::string& s) {
  uint32_t h = 2166136261u;
  for (unsigned char c : s) h = (h ^ c) * 16777619u;
  return h;
}

struct Args {
  std::string model = "raftstereo-sceneflow";
  int batch = 8, steps = 10, warmup = 3, nproc = 0, height = 480, width = 640;
};

int run_rank(const Args& a) {
  sa::dist::DistEnv env = sa::dist::env_from_environment();
  try {
    const int dev = env.local_rank;
    sa::dist::Communicator comm(env, dev);
    sa::EngineConfig cfg;
    cfg.model = a.model;
    cfg.height = a.height;
    cfg.width = a.width;
    cfg.batch = a.batch;
    cfg.device = dev;
    // Every rank runs rank 0's tactic plan: rank 0 builds (tuning each conv shape), exports the entries its engine
    // launches (from the process plan, so this works with plan files disabled), broadcasts those bytes over RCCL,
    // and the other ranks merge them into their tactic table and PIN it (a stale local plan file cannot override a
    // broadcast entry) before building.  Every rank's launched-tactic digest is compared (min == max over ranks).
    hipStream_t bs = nullptr;
    HIP_CHECK(hipStreamCreateWithFlags(&bs, hipStreamNonBlocking));
    std::unique_ptr<sa::StereoEngine> eng;
    std::string plan;
    const std::string tmp = "/tmp/sa_plan_rank" + std::to_string(env.rank) + "_" + std::to_string(getpid());
    if (env.rank == 0) {
      eng = sa::StereoEngine::create(cfg);
      if (sa::conv_plan_save(tmp, eng->plan_keys()) == 0) plan = read_file(tmp);
      std::remove(tmp.c_str());
    }
    comm.broadcast_bytes(plan, 0, bs);
    if (env.rank != 0) {
      if (!plan.empty()) {
        {
          std::ofstream f(tmp, std::ios::binary);
          f.write(plan.data(), (std::streamsize)plan.size());
        }
        sa::conv_plan_load(tmp);
        std::remove(tmp.c_str());
        sa::conv_plan_pin(true);
      }
      eng = sa::StereoEngine::create(cfg);
      sa::conv_plan_pin(false);
    }
    const double ph = (double)fnv32(sa::conv_plan_digest(eng->plan_keys()));
    const bool plans_same = comm.allreduce_max(ph, bs) == -comm.allreduce_max(-ph, bs);
    HIP_CHECK(hipStreamDestroy(bs));
    // The workload of bench.py's step: this rank's B pairs sit in PINNED host memory and are copied H2D every step on
    // a copy stream (issued one step ahead into ping-pong device slots, under the previous step's frame graph), and
    // every frame's point cloud is reprojected inside the frame graph into a per-rank device buffer (kept local)
    const size_t img = (size_t)a.batch * a.height * a.width * 3;
    const size_t npix = (size_t)a.batch * a.height * a.width;
    uint8_t *hl = nullptr, *hr = nullptr;
    HIP_CHECK(hipHostMalloc((void**)&hl, img, hipHostMallocDefault));
    HIP_CHECK(hipHostMalloc((void**)&hr, img, hipHostMallocDefault));
    std::mt19937 rng(1234 + env.rank);
    for (size_t i = 0; i < img; ++i) hl[i] = (uint8_t)(rng() & 0xff);
    for (size_t i = 0; i < img; ++i) hr[i] = hl[(i + 3 * 7) % img];  // shifted copy: a non-trivial pair
    const float Q[16] = {1, 0, 0, -a.width / 2.f, 0, 1, 0, -a.height / 2.f, 0, 0, 0, 500.f, 0, 0, 1 / 60.f, 0};
    eng->set_Q(Q);
    uint8_t *dl[2] = {}, *dr[2] = {};
    float* cloud[2] = {};
    hipEvent_t ready[2], freed[2];
    for (int k = 0; k < 2; ++k) {
      HIP_CHECK(hipMalloc(&dl[k], img));
      HIP_CHECK(hipMalloc(&dr[k], img));
      HIP_CHECK(hipMalloc(&cloud[k], npix * 24));
      HIP_CHECK(hipEventCreateWithFlags(&ready[k], hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&freed[k], hipEventDisableTiming));
    }
    hipStream_t cs = eng->copy_stream();
    hipStream_t es = eng->stream();
    sa::dist::DataParallelRunner dp(eng.get(), &comm);
    long issued = 0, taken = 0;
    bool used[2] = {false, false};
    auto prefetch = [&] {  // H2D of the next step's inputs into slot issued % 2, after that slot's last frame
      const int k = (int)(issued++ % 2);
      if (used[k]) HIP_CHECK(hipStreamWaitEvent(cs, freed[k], 0));
      HIP_CHECK(hipMemcpyAsync(dl[k], hl, img, hipMemcpyHostToDevice, cs));
      HIP_CHECK(hipMemcpyAsync(dr[k], hr, img, hipMemcpyHostToDevice, cs));
      HIP_CHECK(hipEventRecord(ready[k], cs));
    };
    const float* out = nullptr;
    auto step = [&] {
      prefetch();
      const int k = (int)(taken++ % 2);
      HIP_CHECK(hipStreamWaitEvent(es, ready[k], 0));
      out = dp.step(dl[k], dr[k], cloud[k]);
      HIP_CHECK(hipEventRecord(freed[k], es));
      used[k] = true;
    };
    prefetch();
    for (int i = 0; i < a.warmup; ++i) step();
    dp.wait();
    HIP_CHECK(hipStreamSynchronize(cs));
    comm.barrier(dp.comm_stream());
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < a.steps; ++i) step();
    dp.wait();
    comm.barrier(dp.comm_stream());
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double dt_min = -comm.allreduce_max(-dt, dp.comm_stream());
    dt = comm.allreduce_max(dt, dp.comm_stream());
    HIP_CHECK(hipStreamSynchronize(cs));
    // sanity: gathered disparity finite (first and last rank's first pixel)
    float probe[2] = {0, 0};
    const size_t frame = (size_t)a.height * a.width;
    HIP_CHECK(hipMemcpy(&probe[0], out, sizeof(float), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(&probe[1], out + (size_t)(env.world * a.batch - 1) * frame, sizeof(float),
                        hipMemcpyDeviceToHost));
    bool finite = probe[0] == probe[0] && probe[1] == probe[1];
    if (env.rank == 0) {
      double fps = (double)env.world * a.batch * a.steps / dt;
      std::printf(
          "{\"metric\": \"%s %dx%d throughput (frames/s, whole job)\", \"value\": %.3f, \"unit\": \"frames/s\", "
          "\"n_gpus\": %d, \"steps\": %d, \"warmup\": %d, \"ms_per_step\": %.3f, \"higher_is_better\": true, "
          "\"scaling\": \"weak\", \"dtype\": \"fp16\", \"data\": \"synthetic\", \"runner\": \"native-rccl\", "
          "\"finite\": %s, \"plans_identical_across_ranks\": %s, \"tuned_shapes_rank0\": %ld, "
          "\"rank_step_ms\": {\"min\": %.3f, \"max\": %.3f}, \"workload\": \"per-step H2D from pinned host (copy "
          "stream, one step ahead) + frame graph with point-cloud reprojection + RCCL all-gather of disparity\", "
          "\"config\": {\"model\": \"%s\", \"global_batch\": %d, \"per_gpu_batch\": %d, "
          "\"parallelism\": \"dp%d\"}}\n",
          a.model.c_str(), a.height, a.width, fps, env.world, a.steps, a.warmup, dt / a.steps * 1e3,
          finite ? "true" : "false", plans_same ? "true" : "false", eng->tuned_shapes(), dt_min / a.steps * 1e3,
          dt / a.steps * 1e3, a.model.c_str(), env.world * a.batch, a.batch, env.world);
      std::fflush(stdout);
    }
    for (int k = 0; k < 2; ++k) {
      HIP_CHECK(hipFree(dl[k]));
      HIP_CHECK(hipFree(dr[k]));
      HIP_CHECK(hipFree(cloud[k]));
      HIP_CHECK(hipEventDestroy(ready[k]));
      HIP_CHECK(hipEventDestroy(freed[k]));
    }
    HIP_CHECK(hipHostFree(hl));
    HIP_CHECK(hipHostFree(hr));
    return finite ? 0 : 3;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "[rank %d] error: %s\n", env.rank, e.what());
    return 2;
  }
}
}  // namespace

int main(int argc, char** argv) {
  Args a;
  for (int i = 1; i < argc; ++i) {
    std::string k = argv[i];
    auto next = [&]() { return i + 1 < argc ? std::string(argv[++i]) : std::string(); };
    if (k == "--model") a.model = next();
    else if (k == "--batch") a.batch = std::atoi(next().c_str());
    else if (k == "--steps") a.steps = std::atoi(next().c_str());
    else if (k == "--warmup") a.warmup = std::atoi(next().c_str());
    else if (k == "--nproc") a.nproc = std::atoi(next().c_str());
    else if (k == "--height") a.height = std::atoi(next().c_str());
    else if (k == "--width") a.width = std::atoi(next().c_str());
    else {
      std::printf("usage: stereo_bench_dp [--nproc N] [--model preset] [--batch B] [--steps K] [--warmup W]\n");
      return k == "-h" || k == "--help" ? 0 : 1;
    }
  }
  if (a.nproc <= 0) return run_rank(a);
  // fork launcher: no HIP call has happened in this process, so children start clean
  if (!std::getenv("MASTER_ADDR")) setenv("MASTER_ADDR", "127.0.0.1", 1);
  if (!std::getenv("SA_DIST_PORT")) setenv("SA_DIST_PORT", std::to_string(29600 + getpid() % 1000).c_str(), 1);
  std::vector<pid_t> kids;
  for (int r = 0; r < a.nproc; ++r) {
    pid_t p = fork();
    if (p == 0) {
      setenv("RANK", std::to_string(r).c_str(), 1);
      setenv("LOCAL_RANK", std::to_string(r).c_str(), 1);
      setenv("WORLD_SIZE", std::to_string(a.nproc).c_str(), 1);
      std::_Exit(run_rank(a));
    }
    if (p < 0) {
      std::perror("fork");
      for (pid_t k : kids) kill(k, SIGTERM);
      return 1;
    }
    kids.push_back(p);
  }
  int rc = 0;
  for (size_t n = 0; n < kids.size(); ++n) {
    int st = 0;
    pid_t p = wait(&st);
    int code = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
    if (code != 0 && rc == 0) {  // one rank failed: stop its peers instead of letting them time out
      rc = code;
      for (pid_t k : kids)
        if (k != p) kill(k, SIGTERM);
    }
  }
  return rc;
}
