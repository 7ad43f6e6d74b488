// CommGroup (see rccl.h).
#include "rccl.h"

#include <stdexcept>
#include <string>

#include "gale/executor.h"

namespace gale {

namespace {
void check_nccl(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}
}  // namespace

CommGroup::CommGroup(const std::vector<int>& devices) : devices_(devices) {
  if (devices_.empty()) throw std::invalid_argument("CommGroup: no devices");
  comms_.resize(devices_.size());
  check_nccl(ncclCommInitAll(comms_.data(), (int)devices_.size(), devices_.data()),
             "ncclCommInitAll");
  streams_.resize(devices_.size());
  for (size_t i = 0; i < devices_.size(); ++i) {
    check_hip(hipSetDevice(devices_[i]), "CommGroup: hipSetDevice");
    check_hip(hipStreamCreateWithFlags(&streams_[i], hipStreamNonBlocking),
              "CommGroup: hipStreamCreate");
  }
}

CommGroup::~CommGroup() {
  for (size_t i = 0; i < devices_.size(); ++i) {
    hipSetDevice(devices_[i]);
    if (streams_[i]) {
      hipStreamSynchronize(streams_[i]);
      hipStreamDestroy(streams_[i]);
    }
    if (comms_[i]) ncclCommDestroy(comms_[i]);
  }
}

void CommGroup::sync() {
  for (size_t i = 0; i < devices_.size(); ++i) {
    check_hip(hipSetDevice(devices_[i]), "CommGroup: hipSetDevice");
    check_hip(hipStreamSynchronize(streams_[i]), "CommGroup: hipStreamSynchronize");
  }
}

void CommGroup::broadcast(const void* send_root, const std::vector<void*>& recv, size_t bytes,
                          int root) {
  if (recv.size() != devices_.size()) throw std::invalid_argument("broadcast: one buffer per rank");
  if (root < 0 || root >= size()) throw std::invalid_argument("broadcast: bad root");
  // one thread drives every device: the per-device calls must be fused in a group
  check_nccl(ncclGroupStart(), "ncclGroupStart");
  for (size_t i = 0; i < devices_.size(); ++i) {
    check_hip(hipSetDevice(devices_[i]), "broadcast: hipSetDevice");
    check_nccl(ncclBroadcast((int)i == root ? send_root : recv[i], recv[i], bytes, ncclUint8, root,
                             comms_[i], streams_[i]),
               "ncclBroadcast");
  }
  check_nccl(ncclGroupEnd(), "ncclGroupEnd");
  sync();
}

void CommGroup::all_reduce_sum_f64(const std::vector<double*>& bufs, size_t count) {
  if (bufs.size() != devices_.size()) throw std::invalid_argument("all_reduce: one buffer per rank");
  check_nccl(ncclGroupStart(), "ncclGroupStart");
  for (size_t i = 0; i < devices_.size(); ++i) {
    check_hip(hipSetDevice(devices_[i]), "all_reduce: hipSetDevice");
    check_nccl(ncclAllReduce(bufs[i], bufs[i], count, ncclFloat64, ncclSum, comms_[i],
                             streams_[i]),
               "ncclAllReduce");
  }
  check_nccl(ncclGroupEnd(), "ncclGroupEnd");
  sync();
}

}  // namespace gale
