// Native RCCL communicator for the data-parallel gradient path.
//
// One process per MI355X; ranks are joined by an ncclUniqueId that Python distributes over the
// bootstrap process group.  Every collective runs on the communicator's OWN high-priority HIP
// stream: it waits (hipStreamWaitEvent) for an event recorded on the caller's current stream when
// the collective is issued -- i.e. right after the gradients of a bucket were produced -- and
// returns a Work whose wait() makes the caller's stream (not the host) wait for completion.  So
// bucket all-reduces over xGMI overlap the rest of the backward pass, and the host never blocks.
// Buffers used by a collective are recorded on the comm stream for the caching allocator (so the stream
// must stay valid until the process ends: it is taken from torch's stream pool, never destroyed).
//
// Failure detection: a watchdog thread tracks every issued collective (its own completion event + issue
// time).  If one is still pending after `timeout_s`, or RCCL reports an asynchronous error, the watchdog
// calls ncclCommAbort -- which makes the stuck RCCL kernels return -- prints which collective hung, and
// (default) terminates the process with exit code 75 so the launcher tears the job down instead of every
// rank blocking forever in a dead ring.  The reference has no such mechanism.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

namespace rt1comm {

#define COMM_HIP_CHECK(x)                                                                          \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        TORCH_CHECK(e_ == hipSuccess, "HIP error ", hipGetErrorString(e_), " at ", #x);           \
    } while (0)
#define COMM_NCCL_CHECK(x)                                                                         \
    do {                                                                                          \
        ncclResult_t r_ = (x);                                                                    \
        TORCH_CHECK(r_ == ncclSuccess, "RCCL error ", ncclGetErrorString(r_), " at ", #x);        \
    } while (0)

ncclDataType_t to_nccl(at::ScalarType t) {
    switch (t) {
        case at::kFloat: return ncclFloat32;
        case at::kBFloat16: return ncclBfloat16;
        case at::kHalf: return ncclFloat16;
        case at::kDouble: return ncclFloat64;
        case at::kInt: return ncclInt32;
        case at::kLong: return ncclInt64;
        case at::kByte: return ncclUint8;
        default: TORCH_CHECK(false, "rt1_comm: unsupported dtype ", t);
    }
    return ncclFloat32;
}

ncclRedOp_t to_op(const std::string& op) {
    if (op == "sum") return ncclSum;
    if (op == "max") return ncclMax;
    if (op == "min") return ncclMin;
    if (op == "avg") return ncclAvg;
    TORCH_CHECK(false, "rt1_comm: unsupported reduction ", op);
    return ncclSum;
}

// Set by a Python atexit hook: objects garbage-collected during interpreter shutdown must not call
// into the HIP runtime / RCCL any more (they may already be torn down).
static bool g_shutdown = false;

// completion handle of one collective
class Work {
  public:
    explicit Work(hipEvent_t ev) : ev_(ev) {}
    ~Work() {
        if (ev_ && !g_shutdown) (void)hipEventDestroy(ev_);
    }
    // make the caller's current stream wait for the collective (host does not block)
    void wait() {
        COMM_HIP_CHECK(hipStreamWaitEvent(c10::hip::getCurrentHIPStream().stream(), ev_, 0));
    }
    bool is_completed() { return hipEventQuery(ev_) == hipSuccess; }
    void synchronize() { COMM_HIP_CHECK(hipEventSynchronize(ev_)); }

  private:
    hipEvent_t ev_;
};

class Communicator {
  public:
    Communicator(const std::string& uid, int world, int rank, int device, double timeout_s = 600.0)
        : world_(world), rank_(rank), dev_(device), timeout_s_(timeout_s) {
        TORCH_CHECK(uid.size() == sizeof(ncclUniqueId), "rt1_comm: unique id must be ", sizeof(ncclUniqueId),
                    " bytes");
        TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "rt1_comm: bad rank/world");
        ncclUniqueId id;
        memcpy(&id, uid.data(), sizeof(id));
        COMM_HIP_CHECK(hipSetDevice(device));
        // a stream from torch's pool: it outlives this object, which matters because the caching allocator
        // later records events on every stream a freed block was used on.  Default priority: the mere existence
        // of a high-priority queue in the process cost the 1-GPU graph step ~1.0 ms even with the communicator
        // idle (90.9-91.1 vs 89.8-90.0 ms, profiles/r6_graph_dp_world1.log); RT1_COMM_STREAM=high opts back in
        const char* sp = std::getenv("RT1_COMM_STREAM");
        const bool high = sp && std::string(sp) == "high";
        stream_ = c10::hip::getStreamFromPool(/*isHighPriority=*/high, (c10::DeviceIndex)device).stream();
        COMM_NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
        if (timeout_s_ > 0) watchdog_ = std::thread([this] { watch(); });
    }
    ~Communicator() {
        stop_watchdog();
        if (!g_shutdown) destroy();
    }

    void destroy() {
        stop_watchdog();
        std::lock_guard<std::mutex> g(comm_mu_);
        if (comm_) {
            if (!aborted_) {
                (void)hipStreamSynchronize(stream_);
                (void)ncclCommDestroy(comm_);
            }
            comm_ = nullptr;
        }
    }

    bool timed_out() const { return aborted_.load(); }
    void set_exit_on_timeout(bool v) { exit_on_timeout_ = v; }
    // test hook: a pending entry that never completes (exercises the timeout path without hanging a GPU)
    void debug_add_stuck_entry(const std::string& what) {
        std::lock_guard<std::mutex> g(mu_);
        pending_.push_back(Pending{nullptr, std::chrono::steady_clock::now(), what});
    }

    std::shared_ptr<Work> all_reduce_(at::Tensor t, const std::string& op) {
        check(t);
        enter(t);
        COMM_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), to_nccl(t.scalar_type()), to_op(op),
                                     comm_, stream_));
        return leave("all_reduce of " + std::to_string(t.numel()) + " elements");
    }

    std::shared_ptr<Work> broadcast_(at::Tensor t, int root) {
        check(t);
        TORCH_CHECK(root >= 0 && root < world_, "rt1_comm: bad root");
        enter(t);
        COMM_NCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), to_nccl(t.scalar_type()), root,
                                     comm_, stream_));
        return leave("broadcast of " + std::to_string(t.numel()) + " elements");
    }

    // several tensors in one RCCL group launch (one fused submission for many small buckets)
    std::shared_ptr<Work> all_reduce_coalesced_(std::vector<at::Tensor> ts, const std::string& op) {
        for (auto& t : ts) check(t);
        TORCH_CHECK(!ts.empty(), "rt1_comm: empty tensor list");
        enter(ts[0]);
        for (size_t i = 1; i < ts.size(); ++i) record(ts[i]);
        COMM_NCCL_CHECK(ncclGroupStart());
        for (auto& t : ts)
            COMM_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), to_nccl(t.scalar_type()),
                                         to_op(op), comm_, stream_));
        COMM_NCCL_CHECK(ncclGroupEnd());
        return leave("coalesced all_reduce of " + std::to_string(ts.size()) + " tensors");
    }

    int rank() const { return rank_; }
    int world() const { return world_; }
    int device() const { return dev_; }

  private:
    void check(const at::Tensor& t) {
        TORCH_CHECK(!aborted_, "rt1_comm: communicator was aborted by the watchdog (a collective timed out)");
        TORCH_CHECK(comm_, "rt1_comm: communicator destroyed");
        TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "rt1_comm: tensors must be contiguous GPU tensors");
        TORCH_CHECK(t.get_device() == dev_, "rt1_comm: tensor on device ", t.get_device(), ", communicator on ", dev_);
    }
    void record(const at::Tensor& t) {
        auto s = c10::hip::getStreamFromExternal(stream_, dev_);
        c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), s);
    }
    // comm stream waits for everything issued so far on the caller's stream
    void enter(const at::Tensor& t) {
        hipEvent_t ev;
        COMM_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        COMM_HIP_CHECK(hipEventRecord(ev, c10::hip::getCurrentHIPStream(dev_).stream()));
        COMM_HIP_CHECK(hipStreamWaitEvent(stream_, ev, 0));
        COMM_HIP_CHECK(hipEventDestroy(ev));   // destruction is deferred by the runtime until the event completes
        record(t);
    }
    std::shared_ptr<Work> leave(const std::string& what) {
        hipEvent_t done, wd;
        COMM_HIP_CHECK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
        COMM_HIP_CHECK(hipEventRecord(done, stream_));
        if (timeout_s_ > 0) {
            COMM_HIP_CHECK(hipEventCreateWithFlags(&wd, hipEventDisableTiming));
            COMM_HIP_CHECK(hipEventRecord(wd, stream_));
            std::lock_guard<std::mutex> g(mu_);
            pending_.push_back(Pending{wd, std::chrono::steady_clock::now(), what});
        }
        return std::make_shared<Work>(done);
    }

    struct Pending {
        hipEvent_t ev;   // nullptr = debug entry that never completes
        std::chrono::steady_clock::time_point t0;
        std::string what;
    };

    void watch() {
        (void)hipSetDevice(dev_);
        while (!stop_) {
            std::this_thread::sleep_for(std::chrono::milliseconds(50));
            std::string stuck;
            double age = 0.0;
            {
                std::lock_guard<std::mutex> g(mu_);
                while (!pending_.empty()) {
                    Pending& p = pending_.front();
                    if (p.ev != nullptr && hipEventQuery(p.ev) == hipSuccess) {
                        (void)hipEventDestroy(p.ev);
                        pending_.pop_front();
                        continue;
                    }
                    age = std::chrono::duration<double>(std::chrono::steady_clock::now() - p.t0).count();
                    if (age > timeout_s_) stuck = p.what;
                    break;
                }
            }
            ncclResult_t async = ncclSuccess;
            {
                std::lock_guard<std::mutex> g(comm_mu_);
                if (comm_ && !aborted_) (void)ncclCommGetAsyncError(comm_, &async);
            }
            if (stuck.empty() && (async == ncclSuccess || async == ncclInProgress)) continue;
            std::string why = !stuck.empty() ? ("collective '" + stuck + "' pending for " + std::to_string(age) +
                                                " s (timeout " + std::to_string(timeout_s_) + " s)")
                                             : std::string("asynchronous RCCL error: ") + ncclGetErrorString(async);
            fprintf(stderr, "[rt1_comm] rank %d/%d: %s -- aborting the communicator\n", rank_, world_, why.c_str());
            fflush(stderr);
            {
                std::lock_guard<std::mutex> g(comm_mu_);
                if (comm_) (void)ncclCommAbort(comm_);
                aborted_ = true;
            }
            if (exit_on_timeout_) {
                fprintf(stderr, "[rt1_comm] rank %d: exiting with code 75\n", rank_);
                fflush(stderr);
                std::_Exit(75);
            }
            return;
        }
    }

    void stop_watchdog() {
        stop_ = true;
        if (watchdog_.joinable() && std::this_thread::get_id() != watchdog_.get_id()) watchdog_.join();
    }

    int world_, rank_, dev_;
    double timeout_s_;
    ncclComm_t comm_ = nullptr;
    hipStream_t stream_ = nullptr;
    std::mutex mu_, comm_mu_;
    std::deque<Pending> pending_;
    std::thread watchdog_;
    std::atomic<bool> stop_{false}, aborted_{false}, exit_on_timeout_{true};
};

py::bytes unique_id() {
    ncclUniqueId id;
    COMM_NCCL_CHECK(ncclGetUniqueId(&id));
    return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
}

int rccl_version() {
    int v = 0;
    COMM_NCCL_CHECK(ncclGetVersion(&v));
    return v;
}

void register_comm(py::module_& m) {
    auto c = m.def_submodule("comm", "native RCCL communicator (own HIP comm stream)");
    c.def("_mark_shutdown", []() { g_shutdown = true; });
    py::module_::import("atexit").attr("register")(c.attr("_mark_shutdown"));
    c.def("unique_id", &unique_id);
    c.def("rccl_version", &rccl_version);
    py::class_<Work, std::shared_ptr<Work>>(c, "Work", py::module_local())
        .def("wait", &Work::wait)
        .def("is_completed", &Work::is_completed)
        .def("synchronize", &Work::synchronize);
    py::class_<Communicator, std::shared_ptr<Communicator>>(c, "Communicator", py::module_local())
        .def(py::init<const std::string&, int, int, int, double>(), py::arg("uid"), py::arg("world"), py::arg("rank"),
             py::arg("device"), py::arg("timeout_s") = 600.0)
        .def("timed_out", &Communicator::timed_out)
        .def("set_exit_on_timeout", &Communicator::set_exit_on_timeout)
        .def("debug_add_stuck_entry", &Communicator::debug_add_stuck_entry)
        .def("all_reduce_", &Communicator::all_reduce_, py::arg("tensor"), py::arg("op") = "sum")
        .def("all_reduce_coalesced_", &Communicator::all_reduce_coalesced_, py::arg("tensors"), py::arg("op") = "sum")
        .def("broadcast_", &Communicator::broadcast_, py::arg("tensor"), py::arg("root") = 0)
        .def("destroy", &Communicator::destroy)
        .def_property_readonly("rank", &Communicator::rank)
        .def_property_readonly("world", &Communicator::world)
        .def_property_readonly("device", &Communicator::device);
}

}  // namespace rt1comm
