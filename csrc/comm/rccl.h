// In-process RCCL communicator over the GPUs of ONE process (single-process multi-GPU serving).
//
// The reference loads one model copy per InferenceBolt task from disk (InferenceBolt.java:48-58).
// gale materialises the packed weights once on the first GPU and broadcasts them over xGMI to
// every other GPU of the process with ncclCommInitAll + a grouped ncclBroadcast (SURVEY.md §5.8:
// one-time, <= 51 MB, per-link bound ~153 GB/s on the point-to-point xGMI mesh). Multi-process
// deployments (one rank per GPU) use torch.distributed's "nccl" (= RCCL) backend instead
// (gale/parallel/weights.py); both end in the same RCCL broadcast kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace gale {

class CommGroup {
 public:
  explicit CommGroup(const std::vector<int>& devices);
  ~CommGroup();
  CommGroup(const CommGroup&) = delete;
  CommGroup& operator=(const CommGroup&) = delete;

  int size() const { return (int)devices_.size(); }
  const std::vector<int>& devices() const { return devices_; }
  // recv[i] (on devices[i]) <- send of rank `root` (its buffer send_root); bytes per rank.
  // send_root may equal recv[root] (in place). Blocks until every device has the data.
  void broadcast(const void* send_root, const std::vector<void*>& recv, size_t bytes, int root);
  // in-place sum over the ranks' fp64 buffers (benchmark counters)
  void all_reduce_sum_f64(const std::vector<double*>& bufs, size_t count);

 private:
  std::vector<int> devices_;
  std::vector<ncclComm_t> comms_;
  std::vector<hipStream_t> streams_;
  void sync();
};

}  // namespace gale
