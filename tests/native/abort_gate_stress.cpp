// Stress test of pdt::AbortGate (csrc/comm/abort_gate.h), host only, built with AddressSanitizer
// by tests/test_comm_gate_cpu.py.  A heap "communicator" stands in for ncclComm_t: the abort
// frees it (as ncclCommAbort does), issuing threads read and write it inside gate.call(), a
// monitor polls it with try_call() and spammer threads call request_abort() repeatedly.  Any call
// that reached the communicator after the abort freed it is a heap-use-after-free that ASan
// reports (non-zero exit); the program also checks that every issuing thread stopped cleanly.
#include "comm/abort_gate.h"

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

struct FakeComm {
  volatile long calls = 0;
  volatile long polls = 0;
  char payload[256];
};

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 200;
  long total_calls = 0, refused = 0;
  for (int r = 0; r < rounds; ++r) {
    FakeComm* comm = new FakeComm();
    std::atomic<int> aborts_run{0};
    pdt::AbortGate gate([&]() {
      aborts_run.fetch_add(1);
      delete comm;  // ncclCommAbort releases the communicator
    });
    std::atomic<bool> stop{false};
    std::atomic<long> calls{0}, refusals{0};
    std::vector<std::thread> th;
    for (int i = 0; i < 3; ++i)  // issuing threads (the autograd thread issues collectives)
      th.emplace_back([&, i]() {
        std::mt19937 rng(r * 7 + i);
        while (true) {
          const bool ran = gate.call([&]() {
            comm->calls = comm->calls + 1;
            comm->payload[rng() % 256] = (char)i;
            if (rng() % 64 == 0) std::this_thread::yield();  // a slow enqueue
          });
          if (!ran) { refusals.fetch_add(1); break; }  // the wrapper would throw here
          calls.fetch_add(1);
        }
      });
    th.emplace_back([&]() {  // monitor: non-blocking polls, drains a pending abort
      while (!stop.load()) {
        gate.try_call([&]() { comm->polls = comm->polls + 1; });
        gate.drain();
        std::this_thread::yield();
      }
    });
    std::mt19937 rng(r);
    std::this_thread::sleep_for(std::chrono::microseconds(rng() % 2000));
    std::vector<std::thread> spam;
    for (int i = 0; i < 3; ++i)  // abort spammers (monitor failure, user abort, error path)
      spam.emplace_back([&]() {
        for (int k = 0; k < 50; ++k) {
          gate.request_abort();
          std::this_thread::yield();
        }
      });
    for (auto& t : spam) t.join();
    for (int i = 0; i < 3; ++i) th[i].join();  // every issuing thread must end (refused)
    stop.store(true);
    th[3].join();
    gate.drain();
    if (aborts_run.load() != 1 || !gate.aborted()) {
      fprintf(stderr, "round %d: abort ran %d times (aborted=%d)\n", r, aborts_run.load(), (int)gate.aborted());
      return 2;
    }
    // teardown after an abort must not touch the freed communicator
    if (gate.finalize([&]() { comm->calls = -1; })) {
      fprintf(stderr, "round %d: finalize ran after the abort\n", r);
      return 3;
    }
    total_calls += calls.load();
    refused += refusals.load();
  }
  // teardown without an abort runs exactly once
  FakeComm* c2 = new FakeComm();
  pdt::AbortGate g2([&]() { delete c2; });
  int fin = 0;
  g2.finalize([&]() { ++fin; delete c2; });
  if (fin != 1 || g2.finalize([&]() { ++fin; }) || fin != 1) return 4;
  printf("OK rounds=%d calls=%ld refused=%ld\n", rounds, total_calls, refused);
  return 0;
}
