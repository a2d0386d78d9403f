// host_exec.cpp -- see host_exec.h.
#include "host_exec.h"

#include <chrono>

#include "keyspace.h"

namespace rbx {

void Future::complete(int r, std::string m) {
    AsyncCallback c;
    void *u;
    {
        std::lock_guard<std::mutex> g(mu);
        rc = r;
        msg = std::move(m);
        done = true;
        c = cb;
        u = user;
    }
    cv.notify_all();
    if (c) c(u, r);  // outside the lock: the callback may wait on or free other futures
}

bool Future::wait(int64_t timeout_ms) {
    std::unique_lock<std::mutex> g(mu);
    if (timeout_ms < 0) {
        cv.wait(g, [&] { return done; });
        return true;
    }
    return cv.wait_for(g, std::chrono::milliseconds(timeout_ms), [&] { return done; });
}

SerialExecutor::~SerialExecutor() {
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable() && th_.get_id() != std::this_thread::get_id()) th_.join();
}

bool SerialExecutor::on_executor_thread() const {
    return started_ && th_.get_id() == std::this_thread::get_id();
}

void SerialExecutor::release_from_inside(SerialExecutor *e) {
    {
        std::lock_guard<std::mutex> g(e->mu_);
        e->stop_ = true;
        e->self_delete_ = true;
    }
    e->th_.detach();  // loop() deletes the executor once the queue is empty
}

std::shared_ptr<Future> SerialExecutor::submit(std::function<int()> fn, AsyncCallback cb, void *user) {
    auto f = std::make_shared<Future>();
    f->cb = cb;
    f->user = user;
    {
        std::lock_guard<std::mutex> g(mu_);
        if (stop_) return nullptr;
        if (!started_) {
            th_ = std::thread([this] { loop(); });
            started_ = true;
        }
        q_.push_back(Task{std::move(fn), f});
        submitted_++;
        // notified under the lock: once it is released the task may run, and a completion
        // callback may release the executor from inside (release_from_inside), which then frees it
        cv_.notify_all();
    }
    return f;
}

void SerialExecutor::drain() {
    std::unique_lock<std::mutex> g(mu_);
    const uint64_t target = submitted_;
    idle_.wait(g, [&] { return completed_ >= target; });
}

void SerialExecutor::loop() {
    for (;;) {
        Task t;
        {
            std::unique_lock<std::mutex> g(mu_);
            cv_.wait(g, [&] { return stop_ || !q_.empty(); });
            if (q_.empty()) {  // stop requested and nothing left
                if (self_delete_) {
                    g.unlock();
                    delete this;  // detached by release_from_inside(); nobody else owns it
                }
                return;
            }
            t = std::move(q_.front());
            q_.pop_front();
        }
        const int rc = t.fn();
        t.fut->complete(rc, rc ? std::string(last_error_message()) : std::string());
        {
            std::lock_guard<std::mutex> g(mu_);
            completed_++;
        }
        idle_.notify_all();
    }
}

}  // namespace rbx
