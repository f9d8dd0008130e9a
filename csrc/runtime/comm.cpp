// Native RCCL communicator + watchdog (see comm.h).  RCCL is the library torch itself loads
// (same soname librccl.so.1), so one RCCL instance serves both.
#include "comm.h"

#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>

namespace tdl {
namespace comm {

namespace {

void check_nccl(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}
void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP ") + what + ": " + hipGetErrorString(e));
}

ncclDataType_t to_nccl(DType d) {
  switch (d) {
    case DType::F32: return ncclFloat32;
    case DType::BF16: return ncclBfloat16;
    case DType::F16: return ncclFloat16;
    case DType::F64: return ncclFloat64;
    case DType::I32: return ncclInt32;
    case DType::I64: return ncclInt64;
    case DType::U8: return ncclUint8;
  }
  throw std::runtime_error("unsupported dtype");
}

ncclRedOp_t to_nccl(Op o) {
  switch (o) {
    case Op::Sum: return ncclSum;
    case Op::Max: return ncclMax;
    case Op::Min: return ncclMin;
    case Op::Prod: return ncclProd;
    case Op::Avg: return ncclAvg;
  }
  throw std::runtime_error("unsupported op");
}

}  // namespace

std::string get_unique_id() {
  ncclUniqueId id;
  check_nccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, sizeof(id.internal));
}

int rccl_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

Communicator::Communicator(const std::string& uid, int rank, int world, int device, double timeout_s)
    : rank_(rank), world_(world), device_(device), timeout_s_(timeout_s) {
  if (uid.size() != sizeof(ncclUniqueId::internal)) throw std::runtime_error("bad ncclUniqueId size");
  if (rank < 0 || rank >= world) throw std::runtime_error("rank out of range");
  check_hip(hipSetDevice(device), "hipSetDevice");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), sizeof(id.internal));
  ncclComm_t c = nullptr;
  check_nccl(ncclCommInitRank(&c, world, id, rank), "ncclCommInitRank");
  comm_ = c;
  check_hip(hipEventCreateWithFlags(&ready_, hipEventDisableTiming), "hipEventCreate");
  thread_ = std::thread([this] { watchdog(); });
}

Communicator::~Communicator() {
  stop_ = true;
  cv_.notify_all();
  if (thread_.joinable()) thread_.join();
  hipSetDevice(device_);
  if (comm_) {
    // let queued collectives finish (bounded by the timeout), then free the communicator
    const auto t0 = std::chrono::steady_clock::now();
    bool done = false;
    while (!done) {
      done = true;
      for (auto& w : works_) done = done && hipEventQuery(w.done) == hipSuccess;
      if (done) break;
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s_)
        break;
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (done && !failed_)
      ncclCommDestroy((ncclComm_t)comm_);
    else
      ncclCommAbort((ncclComm_t)comm_);
    comm_ = nullptr;
  }
  for (auto& w : works_) hipEventDestroy(w.done);
  for (auto e : free_events_) hipEventDestroy(e);
  for (auto e : parked_events_) hipEventDestroy(e);
  for (auto e : graph_events_) hipEventDestroy(e);
  if (ready_) hipEventDestroy(ready_);
}

hipEvent_t Communicator::take_event() {
  if (!free_events_.empty()) {
    hipEvent_t e = free_events_.back();
    free_events_.pop_back();
    return e;
  }
  hipEvent_t e;
  check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  return e;
}

template <class F>
uint64_t Communicator::enqueue(const char* name, hipStream_t producer, hipStream_t comm, F&& issue) {
  std::lock_guard<std::mutex> g(mu_);
  if (failed_ || !comm_) throw std::runtime_error("RCCL communicator failed: " + error_);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  check_hip(hipStreamIsCapturing(producer, &cap), "hipStreamIsCapturing");
  if (cap == hipStreamCaptureStatusActive) {
    // HIP-graph capture: fresh events (graph nodes reference them), comm stream forked into the
    // capture by the wait, collective captured, completion event for the consumer's wait
    hipEvent_t rdy, done;
    check_hip(hipEventCreateWithFlags(&rdy, hipEventDisableTiming), "hipEventCreate");
    graph_events_.push_back(rdy);
    check_hip(hipEventCreateWithFlags(&done, hipEventDisableTiming), "hipEventCreate");
    graph_events_.push_back(done);
    check_hip(hipEventRecord(rdy, producer), "hipEventRecord (capture)");
    check_hip(hipStreamWaitEvent(comm, rdy, 0), "hipStreamWaitEvent (capture)");
    check_nccl(issue((ncclComm_t)comm_), name);
    check_hip(hipEventRecord(done, comm), "hipEventRecord (capture)");
    const uint64_t t = next_ticket_++;
    graph_works_.emplace_back(t, done);
    return t;
  }
  if (cap != hipStreamCaptureStatusNone)
    throw std::runtime_error("RCCL collective on a stream whose capture was invalidated");
  recycle_graph_events();
  if (producer != comm) {
    check_hip(hipEventRecord(ready_, producer), "hipEventRecord");
    check_hip(hipStreamWaitEvent(comm, ready_, 0), "hipStreamWaitEvent");
  }
  check_nccl(issue((ncclComm_t)comm_), name);
  hipEvent_t done = take_event();
  check_hip(hipEventRecord(done, comm), "hipEventRecord");
  const uint64_t t = next_ticket_++;
  works_.push_back(Work{t, done, std::chrono::steady_clock::now(), name});
  return t;
}

uint64_t Communicator::all_reduce(const void* send, void* recv, size_t count, DType dt, Op op,
                                  hipStream_t producer, hipStream_t comm, const char* name) {
  return enqueue(name, producer, comm, [&](ncclComm_t c) {
    return ncclAllReduce(send, recv, count, to_nccl(dt), to_nccl(op), c, comm);
  });
}

uint64_t Communicator::broadcast(const void* send, void* recv, size_t count, DType dt, int root,
                                 hipStream_t producer, hipStream_t comm) {
  return enqueue("broadcast", producer, comm, [&](ncclComm_t c) {
    return ncclBroadcast(send, recv, count, to_nccl(dt), root, c, comm);
  });
}

uint64_t Communicator::reduce_scatter(const void* send, void* recv, size_t count, DType dt, Op op,
                                      hipStream_t producer, hipStream_t comm) {
  return enqueue("reduce_scatter", producer, comm, [&](ncclComm_t c) {
    return ncclReduceScatter(send, recv, count, to_nccl(dt), to_nccl(op), c, comm);
  });
}

uint64_t Communicator::all_gather(const void* send, void* recv, size_t count, DType dt,
                                  hipStream_t producer, hipStream_t comm) {
  return enqueue("all_gather", producer, comm, [&](ncclComm_t c) {
    return ncclAllGather(send, recv, count, to_nccl(dt), c, comm);
  });
}

// A finished capture's events: stream capture turned their record / wait pairs into graph edges,
// so no graph node references them — the next eager collective (or tracked replay) returns them
// to the free list instead of keeping two per captured collective for the communicator's life.
// Tickets of a finished capture are only waited on inside that capture, so its list is dropped.
void Communicator::recycle_graph_events() {
  if (graph_events_.empty() && graph_works_.empty()) return;
  free_events_.insert(free_events_.end(), graph_events_.begin(), graph_events_.end());
  graph_events_.clear();
  graph_works_.clear();
}

uint64_t Communicator::track(const char* name, hipStream_t comm) {
  std::lock_guard<std::mutex> g(mu_);
  if (failed_ || !comm_) throw std::runtime_error("RCCL communicator failed: " + error_);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(comm, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone)
    recycle_graph_events();
  hipEvent_t done = take_event();
  check_hip(hipEventRecord(done, comm), "hipEventRecord");
  const uint64_t t = next_ticket_++;
  works_.push_back(Work{t, done, std::chrono::steady_clock::now(), name});
  return t;
}

void Communicator::wait(uint64_t ticket, hipStream_t consumer) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& w : graph_works_) {
    if (w.first == ticket) {
      check_hip(hipStreamWaitEvent(consumer, w.second, 0), "hipStreamWaitEvent");
      return;
    }
  }
  for (auto& w : works_) {
    if (w.ticket == ticket) {
      check_hip(hipStreamWaitEvent(consumer, w.done, 0), "hipStreamWaitEvent");
      return;
    }
  }
  // not outstanding: already completed and retired by the watchdog
}

void Communicator::synchronize() {
  std::vector<hipEvent_t> evs;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& w : works_) evs.push_back(w.done);
    ++sync_pins_;  // none of these handles is recycled until we are done with them
  }
  for (auto e : evs) {
    if (failed_) break;
    hipEventSynchronize(e);
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    if (--sync_pins_ == 0) {
      free_events_.insert(free_events_.end(), parked_events_.begin(), parked_events_.end());
      parked_events_.clear();
    }
  }
  if (failed_) throw std::runtime_error("RCCL communicator failed: " + error());
}

std::string Communicator::error() const {
  std::lock_guard<std::mutex> g(mu_);
  return error_;
}

int Communicator::rccl_count() const {
  std::lock_guard<std::mutex> g(mu_);
  if (!comm_) throw std::runtime_error("RCCL communicator failed: " + error_);
  int n = 0;
  check_nccl(ncclCommCount((ncclComm_t)comm_, &n), "ncclCommCount");
  return n;
}

int Communicator::rccl_rank() const {
  std::lock_guard<std::mutex> g(mu_);
  if (!comm_) throw std::runtime_error("RCCL communicator failed: " + error_);
  int r = -1;
  check_nccl(ncclCommUserRank((ncclComm_t)comm_, &r), "ncclCommUserRank");
  return r;
}

int Communicator::rccl_device() const {
  std::lock_guard<std::mutex> g(mu_);
  if (!comm_) throw std::runtime_error("RCCL communicator failed: " + error_);
  int d = -1;
  check_nccl(ncclCommCuDevice((ncclComm_t)comm_, &d), "ncclCommCuDevice");
  return d;
}

size_t Communicator::outstanding() const {
  std::lock_guard<std::mutex> g(mu_);
  return works_.size();
}

void Communicator::abort(const std::string& why) {
  std::lock_guard<std::mutex> g(mu_);  // no collective is being enqueued meanwhile
  bool expected = false;
  if (!failed_.compare_exchange_strong(expected, true)) return;
  error_ = why;
  if (comm_) {
    hipSetDevice(device_);
    ncclCommAbort((ncclComm_t)comm_);  // unblocks RCCL kernels waiting on peers
    comm_ = nullptr;
  }
}

void Communicator::watchdog() {
  hipSetDevice(device_);
  while (!stop_) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait_for(lk, std::chrono::milliseconds(50), [this] { return stop_.load(); });
    }
    if (stop_ || failed_) continue;
    std::string why;
    {
      std::lock_guard<std::mutex> g(mu_);
      // retire completed collectives in issue order (the comm stream is in-order)
      while (!works_.empty() && hipEventQuery(works_.front().done) == hipSuccess) {
        (sync_pins_ > 0 ? parked_events_ : free_events_).push_back(works_.front().done);
        works_.pop_front();
      }
      if (!works_.empty()) {
        const double age = std::chrono::duration<double>(std::chrono::steady_clock::now() -
                                                         works_.front().t0).count();
        if (age > timeout_s_)
          why = "collective '" + works_.front().name + "' (ticket " +
                std::to_string(works_.front().ticket) + ") not complete after " +
                std::to_string((int)age) + " s on rank " + std::to_string(rank_);
      }
      if (why.empty() && comm_) {
        ncclResult_t ar = ncclSuccess;
        if (ncclCommGetAsyncError((ncclComm_t)comm_, &ar) == ncclSuccess && ar != ncclSuccess &&
            ar != ncclInProgress)
          why = std::string("RCCL async error on rank ") + std::to_string(rank_) + ": " +
                ncclGetErrorString(ar);
      }
    }
    if (!why.empty()) abort(why);
  }
}

}  // namespace comm
}  // namespace tdl
