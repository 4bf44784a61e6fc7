// lastwords.cpp -- a measured result that outlives the process's end.  A multi-rank bench run holds
// its finished line while the north_star size sweep runs; if the process is then ended from
// outside (torch.distributed.run sends SIGTERM to every rank when one rank dies, a time limit
// sends SIGTERM/SIGINT/SIGHUP) or dies by itself (a GPU memory fault ends in abort(); a crash), a
// Python-level handler cannot help: the main thread may be blocked inside a collective or a device
// wait, and an abort never returns to the interpreter.  This handler writes the registered line
// with write(2) -- async-signal-safe -- once, then restores the handler that was there before and
// re-raises, so faulthandler's dump and the default action still follow.
//
// Two static line buffers: dpwa_last_words_set fills the inactive one and then publishes it with
// one atomic store, so a signal arriving mid-update writes the previous, complete line.  The
// normal end prints the line through dpwa_last_words_flush: the line is written exactly once,
// by whichever of the flush and a signal claims it first (a handler that finds the flush writing
// on another thread waits for it, up to 2 s, before the process goes).
#include <pthread.h>
#include <signal.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <csignal>
#include <cstring>
#include <mutex>

#include "common.hpp"

namespace {

constexpr size_t kLineCap = 16384;
constexpr int kSignals[] = {SIGTERM, SIGINT, SIGHUP, SIGABRT, SIGSEGV, SIGBUS, SIGFPE, SIGILL};

struct Line {
    char buf[kLineCap];
    size_t len;
};

Line g_lines[2];
std::atomic<Line *> g_active{nullptr};      // nullptr: nothing to write
std::atomic<int> g_fd{-1};
std::atomic<int> g_state{0};                // 0 armed, 1 being written (by the flush), 2 written
int g_next = 0;                             // the buffer the next set fills (setter side only)
std::mutex g_set_mu;
bool g_installed = false;
struct sigaction g_prev[sizeof(kSignals) / sizeof(kSignals[0])];

int slot_of(int sig)
{
    for (size_t i = 0; i < sizeof(kSignals) / sizeof(kSignals[0]); ++i)
        if (kSignals[i] == sig) return (int)i;
    return -1;
}

void write_all(int fd, const Line *l)
{
    const char *p = l->buf;
    size_t left = l->len;
    while (left) {
        const ssize_t w = write(fd, p, left);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) break;
        p += w;
        left -= (size_t)w;
    }
}

// Claims the line (state 0 -> 1), writes it, marks it written; false when it was claimed before.
bool write_once()
{
    Line *l = g_active.load(std::memory_order_acquire);
    const int fd = g_fd.load(std::memory_order_relaxed);
    int armed = 0;
    if (!l || fd < 0 || !g_state.compare_exchange_strong(armed, 1)) return false;
    write_all(fd, l);
    g_state.store(2);
    return true;
}

void on_signal(int sig)
{
    const int saved = errno;
    if (!write_once()) {
        // the flush may be writing on another thread (it blocks these signals on its own): let it
        // finish before the previous handler ends the process
        for (int i = 0; i < 2000 && g_state.load() == 1; ++i) {
            struct timespec ts = {0, 1000000};
            nanosleep(&ts, nullptr);
        }
    }
    const int i = slot_of(sig);
    if (i >= 0) sigaction(sig, &g_prev[i], nullptr);   // the previous handler (or the default) ...
    errno = saved;
    raise(sig);                                        // ... runs once this one returns
}

bool install()
{
    for (size_t i = 0; i < sizeof(kSignals) / sizeof(kSignals[0]); ++i) {
        struct sigaction sa;
        memset(&sa, 0, sizeof(sa));
        sa.sa_handler = on_signal;
        sigemptyset(&sa.sa_mask);
        sa.sa_flags = SA_RESTART;
        if (sigaction(kSignals[i], &sa, &g_prev[i]) != 0) return false;
        // an ignored signal (SIGHUP under nohup) does not end the process: it stays ignored, or
        // the line would be written for a run that goes on
        if (!(g_prev[i].sa_flags & SA_SIGINFO) && g_prev[i].sa_handler == SIG_IGN)
            sigaction(kSignals[i], &g_prev[i], nullptr);
    }
    return true;
}

}  // namespace

extern "C" int dpwa_last_words_set(int fd, const char *line, int64_t len)
{
    if (len < 0 || (len > 0 && (!line || fd < 0)) || (size_t)len > kLineCap)
        return dpwa::set_error(DPWA_ERR_ARG, "dpwa_last_words_set: %lld bytes (at most %zu) to fd %d",
                               (long long)len, kLineCap, fd);
    std::lock_guard<std::mutex> g(g_set_mu);
    if (len == 0) {
        g_active.store(nullptr, std::memory_order_release);
        return DPWA_OK;
    }
    if (!g_installed) {
        if (!install()) return dpwa::set_error(DPWA_ERR_STATE, "dpwa_last_words_set: sigaction: %s", strerror(errno));
        g_installed = true;
    }
    Line &l = g_lines[g_next];
    memcpy(l.buf, line, (size_t)len);
    l.len = (size_t)len;
    g_fd.store(fd, std::memory_order_relaxed);
    g_active.store(&l, std::memory_order_release);
    g_next ^= 1;
    return DPWA_OK;
}

extern "C" int dpwa_last_words_flush(int *wrote)
{
    sigset_t block, old;
    sigemptyset(&block);
    for (int sig : kSignals) sigaddset(&block, sig);
    pthread_sigmask(SIG_BLOCK, &block, &old);      // no handler on this thread mid-write
    const bool w = write_once();
    pthread_sigmask(SIG_SETMASK, &old, nullptr);
    if (wrote) *wrote = w ? 1 : 0;
    return DPWA_OK;
}

extern "C" int dpwa_last_words_written(int *written)
{
    if (!written) return dpwa::set_error(DPWA_ERR_ARG, "dpwa_last_words_written: NULL argument");
    *written = g_state.load() == 2 ? 1 : 0;
    return DPWA_OK;
}
