// Host memory read bandwidth by thread count (is a host stage memory-bound on this box?).
// g++ -O2 -pthread scripts/probe_hostbw.cpp -o /tmp/probe_hostbw && /tmp/probe_hostbw
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>
#include <cstdint>
int main(){
  size_t N = 256u << 20; std::vector<uint64_t> a(N/8, 1);
  for (int nt : {1, 2, 4, 8, 16, 1, 16}) {
    std::vector<uint64_t> s(nt*8);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back([&, t]{ uint64_t x = 0; size_t lo = a.size()*t/nt, hi = a.size()*(t+1)/nt; for (size_t i = lo; i < hi; i += 16) x += a[i]; s[t*8] = x; });
    for (auto& x : th) x.join();
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now()-t0).count();
    printf("nt %d %.1f ms %.1f GB/s (lines)\n", nt, dt*1e3, N/dt/1e9);
  }
}
