// host_exec.h -- per-context serial executor behind the asynchronous entry points of
// include/rbx.h (the RHyperLogLogAsync / RFuture surface, M/api/RHyperLogLogAsync.java:37-70).
// Plain C++17, no HIP: tests/c/keyspace_test.cpp runs it under ASan/UBSan and TSan.
//
// Calls submitted to one context run one after another on the executor's thread, in submission
// order (a context serializes its batches, include/rbx.h), each completing its Future: the call's
// return code, its error message, then the optional C callback (a JVM binds it as an FFM upcall
// that completes a CompletableFuture).
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

namespace rbx {

typedef void (*AsyncCallback)(void *user, int rc);

struct Future {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    int rc = 0;
    std::string msg;  // rbx_last_error() of the call when rc != 0
    AsyncCallback cb = nullptr;
    void *user = nullptr;

    void complete(int r, std::string m);
    // true when done within timeout_ms (< 0: wait for ever)
    bool wait(int64_t timeout_ms);
};

class SerialExecutor {
public:
    SerialExecutor() = default;
    SerialExecutor(const SerialExecutor &) = delete;
    SerialExecutor &operator=(const SerialExecutor &) = delete;
    ~SerialExecutor();  // runs what is queued, then joins the thread

    // nullptr once the executor is stopping (the caller reports the context as shut down)
    std::shared_ptr<Future> submit(std::function<int()> fn, AsyncCallback cb, void *user);
    void drain();  // returns once everything submitted so far has completed
    // true on the executor's own thread (a completion callback)
    bool on_executor_thread() const;
    // Stop from the executor's own thread: later submits are refused, what is queued still runs,
    // and the executor frees itself when its thread leaves the loop (it cannot join itself).
    // The caller gives up ownership.
    static void release_from_inside(SerialExecutor *e);

private:
    struct Task {
        std::function<int()> fn;
        std::shared_ptr<Future> fut;
    };
    void loop();

    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Task> q_;
    bool stop_ = false;
    bool started_ = false;
    bool self_delete_ = false;
    uint64_t submitted_ = 0, completed_ = 0;
    std::condition_variable idle_;
    std::thread th_;
};

}  // namespace rbx
