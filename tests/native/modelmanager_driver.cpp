// modelmanager_driver.cpp -- TEST INFRASTRUCTURE: the C++ ModelManager
// (crossbow_amd/host/ModelManager.hpp) driving the library on the GPU the way
// Crossbow's ResultCollector drives the Java one: registration, one barrier
// per clock with autotuning on a scripted throughput monitor, checkpoints by
// clock.  Checks the replica count after each autotune decision, the
// checkpoint versions, and the first step bit for bit against the oracle.
// Built by scripts/build_host_harness.sh; run by tests/test_gpu_host.py.
#include <sys/stat.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <unistd.h>

#include "ModelManager.hpp"
#include "sma_oracle.h"

#define EXPECT(cond)                                                                      \
  do {                                                                                    \
    if (!(cond)) {                                                                        \
      std::fprintf(stderr, "%s:%d expectation failed: %s\n", __FILE__, __LINE__, #cond); \
      std::exit(1);                                                                       \
    }                                                                                     \
  } while (0)

int main() {
  using crossbow::check;
  const int n = 4099, R = 2;
  const float alpha = 0.1f, momentum = 0.9f;
  cbx_context *gpu = nullptr;
  int dev = 0;
  check(cbx_init(&gpu, &dev, 1), "init");

  // Model.GPURegister / SolverConf.GPURegister
  std::vector<float> z0(n);
  cbo_fill_normal(z0.data(), n, CBO_SEED ^ CBO_BUF_Z, 0.05f, nullptr);
  const int shape[1] = {n};
  check(cbx_set_model(gpu, 1, 4 * n), "setModel");
  check(cbx_set_model_variable(gpu, 0, 1, 1, shape, 4 * n), "setModelVariable");
  check(cbx_set_model_variable_buffer(gpu, 0, 1, z0.data()), "setModelVariableBuffer");
  check(cbx_set_model_work_per_clock(gpu, 2), "setModelWorkPerClock");
  check(cbx_set_update_model_type(gpu, CBX_UPDATE_SMA), "setUpdateModelType");
  check(cbx_set_learning_rate_decay_policy_fixed(gpu, 0.05f), "setLearningRateDecayPolicyFixed");
  check(cbx_set_momentum(gpu, momentum, 0), "setMomentum");
  check(cbx_set_eamsgd_alpha(gpu, alpha), "setEamsgdAlpha");

  char dir[] = "/tmp/cbx_modelmanagerXXXXXX";
  EXPECT(mkdtemp(dir) != nullptr);
  crossbow::SystemConf conf;
  conf.replicasPerGpu = R;
  conf.wpc = 2;
  conf.checkpointInterval = 3;  // tasks -> rounded up to 4 -> every 2 clocks
  conf.checkpointDirectory = dir;
  conf.autotuneModels = true;
  conf.autotuneInterval = 2;
  crossbow::ModelManager manager(gpu, conf);
  EXPECT(manager.checkpointStep() == 2);
  // Throughput readings at the autotune points (barriers 2, 4, 6): first
  // reading counts as an improvement, +50 % improves, -6.7 % does not.
  const double readings[] = {100.0, 150.0, 140.0};
  int reads = 0;
  manager.setPerformanceMonitor([&] { return readings[reads++]; });
  manager.GPURegister();
  EXPECT(cbx_num_replicas(gpu) == R);

  // Oracle for the first barrier: every replica starts as theModel, no task
  // wrote a snapshot (s = 0), last = 0.
  std::vector<float> z = z0, last(n, 0.0f), scratch(2 * n);
  std::vector<std::vector<float>> s(R, std::vector<float>(n, 0.0f)), w(R, z0);
  float *zp = z.data(), *lp = last.data();
  float *sp[R], *wp[R];
  for (int i = 0; i < R; ++i) {
    sp[i] = s[i].data();
    wp[i] = w[i].data();
  }
  int locked[R] = {1, 1}, copy[R] = {0, 0};
  cbo_sma_fma(1, R, n, alpha, momentum, &zp, &lp, sp, wp, locked, copy, 0, scratch.data());

  const int expect_replicas[] = {2, 3, 3, 4, 4, 3, 3, 3};  // after clocks 1..8
  for (int clock = 1; clock <= 8; ++clock) {
    EXPECT(manager.trySynchronise(clock));
    EXPECT(cbx_num_replicas(gpu) == expect_replicas[clock - 1]);
    if (clock == 1) {
      std::vector<float> got(n);
      check(cbx_base_read(gpu, 0, CBX_BUF_DATA, got.data(), 4 * (size_t)n), "base_read");
      EXPECT(std::memcmp(got.data(), z.data(), 4 * (size_t)n) == 0);
      for (int i = 0; i < R; ++i) {
        check(cbx_replica_read(gpu, i, CBX_BUF_DATA, got.data(), 4 * (size_t)n), "replica_read");
        EXPECT(std::memcmp(got.data(), w[i].data(), 4 * (size_t)n) == 0);
      }
    }
    EXPECT(manager.checkpoint(clock) == (clock % 2 == 0));
  }
  EXPECT(reads == 3 && !manager.autotuning());
  for (int v = 1; v <= 4; ++v) {
    char path[512];
    std::snprintf(path, sizeof path, "%s/%06d/gpu-00-theModel-data.dat", dir, v);
    struct stat st;
    EXPECT(stat(path, &st) == 0 && st.st_size == 4 * n);
  }
  // Checkpoint 2 (clock 4, after the second add) holds 4 replicas; checkpoint
  // 3 (clock 6, after the delete) holds 3.
  {
    char path[512];
    struct stat st;
    std::snprintf(path, sizeof path, "%s/000002/gpu-00-replica-003-data.dat", dir);
    EXPECT(stat(path, &st) == 0);
    std::snprintf(path, sizeof path, "%s/000003/gpu-00-replica-003-data.dat", dir);
    EXPECT(stat(path, &st) != 0);
  }
  // A library error surfaces as CbxError with the library's message.
  bool threw = false;
  try {
    check(cbx_replica_lock(gpu, 99), "replica_lock");
  } catch (const crossbow::CbxError &e) {
    threw = e.code() == CBX_ERR_INVALID && std::strstr(e.what(), "out of range") != nullptr;
  }
  EXPECT(threw);
  check(cbx_free(gpu), "free");
  std::printf("modelmanager_driver: ok\n");
  std::fflush(stdout);
  _exit(0);
}
