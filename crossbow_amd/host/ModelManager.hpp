// ModelManager.hpp -- the barrier-side caller of the SMA path in C++, over the
// C-ABI of include/crossbow_sma.h.
//
// Restates the GPU body of Crossbow's Java ModelManager
// (src/main/java/uk/ac/imperial/lsds/crossbow/model/ModelManager.java) for
// hosts without a JVM, with the same method names and argument meaning:
//   * GPURegister          :355-358   setModelManager(replicas per GPU, sync model)
//   * trySynchronise(clock):293-353   lockAny -> synchronise(0, clock, autotune(), false) -> unlockAny
//   * autotune             :257-274   every `interval` barriers while autotuning: +1 if the
//                                     throughput improved by more than `threshold`, else -1
//                                     once and autotuning ends
//   * hasThroughputImproved:238-255
//   * checkpoint(clock)    :276-286   every checkpointStep clocks, the step being the
//                                     checkpoint interval in tasks rounded up to whole
//                                     clocks (:73-80)
// Settings are the SystemConf / ModelConf ones the Java class reads
// (SystemConf.java:209-231 defaults: no checkpoints, autotuning off,
// threshold 0.1, interval 1; wpc from ModelConf).
//
// Errors: a negative status from the library throws CbxError carrying
// cbx_last_error(); the Java class's own exceptions (null monitor, bad
// configuration) are std::logic_error.  Header-only; link libcrossbow_sma.
#pragma once

#include <functional>
#include <stdexcept>
#include <string>
#include <utility>

#include "crossbow_sma.h"

namespace crossbow {

class CbxError : public std::runtime_error {
 public:
  CbxError(int code, const std::string &what) : std::runtime_error(what), code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

inline int check(int rc, const char *call) {
  if (rc < 0) throw CbxError(rc, std::string(call) + ": " + cbx_last_error());
  return rc;
}

struct SystemConf {
  int replicasPerGpu = 1;                // --number-of-gpu-models
  int synchronisationModel = CBX_SYNC_BSP;  // --synchronisation-model
  int wpc = 1;                           // ModelConf --wpc
  long checkpointInterval = 0;           // tasks; 0 = never
  std::string checkpointDirectory;       // --checkpoint-directory
  bool autotuneModels = false;           // --autotune-models
  double autotuneThreshold = 0.1;
  int autotuneInterval = 1;
};

class ModelManager {
 public:
  ModelManager(cbx_context *gpu, SystemConf conf) : gpu_(gpu), conf_(std::move(conf)) {
    if (conf_.wpc <= 0) throw std::logic_error("error: work per clock must be positive");
    if (conf_.autotuneInterval <= 0) throw std::logic_error("error: autotune interval must be positive");
    long step = conf_.checkpointInterval;
    while (step % conf_.wpc != 0) ++step;
    checkpointStep_ = step / conf_.wpc;
    autotuning_ = conf_.autotuneModels;
  }

  // PerformanceMonitor.getCurrentThroughput(0)
  ModelManager &setPerformanceMonitor(std::function<double()> monitor) {
    monitor_ = std::move(monitor);
    return *this;
  }

  void GPURegister() {
    check(cbx_set_model_manager(gpu_, conf_.replicasPerGpu, conf_.synchronisationModel), "setModelManager");
  }

  bool trySynchronise(int clock) {
    check(cbx_lock_any(gpu_), "lockAny");
    check(cbx_synchronise(gpu_, 0, clock, autotune(), 0), "synchronise");
    check(cbx_unlock_any(gpu_), "unlockAny");
    return true;
  }

  bool checkpoint(int clock) {
    if (checkpointStep_ <= 0 || clock % checkpointStep_ != 0) return false;
    if (conf_.checkpointDirectory.empty())
      throw std::logic_error("error: checkpoint interval set without a checkpoint directory");
    check(cbx_checkpoint_model(gpu_, conf_.checkpointDirectory.c_str()), "checkpointModel");
    return true;
  }

  int autotune() {
    if (conf_.autotuneModels && autotuning_ && (++step_ % conf_.autotuneInterval) == 0) {
      if (hasThroughputImproved()) return 1;
      autotuning_ = false;
      return -1;
    }
    return 0;
  }

  long checkpointStep() const { return checkpointStep_; }
  bool autotuning() const { return autotuning_; }

 private:
  bool hasThroughputImproved() {
    if (!monitor_) throw std::logic_error("error: performance monitor is null");
    const double current = monitor_();
    const double delta = (throughput_ == 0) ? 1.0 : (current - throughput_) / throughput_;
    throughput_ = current;
    return delta > conf_.autotuneThreshold;
  }

  cbx_context *gpu_;
  SystemConf conf_;
  long checkpointStep_ = 0;
  bool autotuning_ = false;
  std::function<double()> monitor_;
  double throughput_ = 0.0;
  long step_ = 0;
};

}  // namespace crossbow
