// Native RCCL communicator with a dedicated comm stream and a watchdog thread (SURVEY §5.8 / N14,
// §5.3).  Torch-free: raw device pointers and hipStream_t; csrc/bindings.cpp adds the tensor glue.
//
//   * one process per GPU; the 128-byte ncclUniqueId is produced by rank 0 (get_unique_id) and
//     distributed by the caller (the Python side uses the torch.distributed store / gloo group);
//   * every collective is enqueued on the caller-supplied comm stream after an event recorded on
//     the producer (compute) stream — no host synchronisation — and returns a ticket; wait(ticket,
//     consumer) makes the consumer stream wait on the collective's completion event;
//   * collectives enqueued while the producer stream is capturing a HIP graph are captured with
//     it (event record / wait nodes fork the comm stream into the capture) and replay with it;
//   * the watchdog polls outstanding collectives (hipEventQuery) and ncclCommGetAsyncError; a
//     collective older than `timeout_s` or an async RCCL error aborts the communicator
//     (ncclCommAbort) and latches an error string the Python side raises on (fail fast instead of
//     hanging every rank).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace tdl {
namespace comm {

enum class DType { F32, BF16, F16, F64, I32, I64, U8 };
enum class Op { Sum, Max, Min, Prod, Avg };

std::string get_unique_id();  // 128 raw bytes
int rccl_version();

class Communicator {
 public:
  Communicator(const std::string& uid, int rank, int world, int device, double timeout_s);
  ~Communicator();
  Communicator(const Communicator&) = delete;
  Communicator& operator=(const Communicator&) = delete;

  uint64_t all_reduce(const void* send, void* recv, size_t count, DType dt, Op op,
                      hipStream_t producer, hipStream_t comm, const char* name = "all_reduce");
  uint64_t broadcast(const void* send, void* recv, size_t count, DType dt, int root,
                     hipStream_t producer, hipStream_t comm);
  // recv holds count elements; send holds count·world
  uint64_t reduce_scatter(const void* send, void* recv, size_t count, DType dt, Op op,
                          hipStream_t producer, hipStream_t comm);
  // send holds count elements; recv holds count·world
  uint64_t all_gather(const void* send, void* recv, size_t count, DType dt, hipStream_t producer,
                      hipStream_t comm);

  // registers the work queued so far on `comm` as an outstanding item (watched like a
  // collective) — fault-injection tests stall the stream and let the watchdog fire without any
  // RCCL operation in flight
  uint64_t track(const char* name, hipStream_t comm);

  // stream-level, no host block (tickets of collectives captured into a HIP graph included)
  void wait(uint64_t ticket, hipStream_t consumer);
  void synchronize();                                  // host waits for every outstanding collective
  std::string error() const;
  bool ok() const { return !failed_.load(); }
  void abort(const std::string& why);
  int rank() const { return rank_; }
  int world() const { return world_; }
  // what RCCL itself reports for this communicator (ncclCommCount / ncclCommUserRank /
  // ncclCommCuDevice) — the bench cross-checks the rank count against its --gpus
  int rccl_count() const;
  int rccl_rank() const;
  int rccl_device() const;
  size_t outstanding() const;

 private:
  struct Work {
    uint64_t ticket;
    hipEvent_t done;
    std::chrono::steady_clock::time_point t0;
    std::string name;
  };
  template <class F>
  uint64_t enqueue(const char* name, hipStream_t producer, hipStream_t comm, F&& issue);
  hipEvent_t take_event();
  void watchdog();

  void* comm_ = nullptr;  // ncclComm_t
  int rank_, world_, device_;
  double timeout_s_;
  hipEvent_t ready_ = nullptr;  // producer → comm ordering event (re-recorded per collective)
  mutable std::mutex mu_;
  std::deque<Work> works_;
  std::vector<hipEvent_t> free_events_;
  // synchronize() waits on snapshotted event handles outside the lock: while any such wait is in
  // progress, retired events are parked here instead of being recycled, so a handle it holds is
  // never re-recorded by a later collective (it would then also wait for that newer work)
  std::vector<hipEvent_t> parked_events_;
  // collectives issued while the producer stream is being captured into a HIP graph: they run
  // at every replay, so they are not watched as outstanding work (ncclCommGetAsyncError still
  // is); their ordering events become graph edges at capture, so they return to the free list at
  // the next eager collective or tracked replay (recycle_graph_events)
  void recycle_graph_events();  // caller holds mu_, no capture in progress
  std::vector<std::pair<uint64_t, hipEvent_t>> graph_works_;
  std::vector<hipEvent_t> graph_events_;
  int sync_pins_ = 0;
  uint64_t next_ticket_ = 1;
  std::atomic<bool> failed_{false};
  std::atomic<bool> stop_{false};
  std::string error_;
  std::condition_variable cv_;
  std::thread thread_;
};

}  // namespace comm
}  // namespace tdl
