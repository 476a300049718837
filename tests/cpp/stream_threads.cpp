// stream_threads.cpp -- the drop-in header (include/smallz4_amd.hpp) under load, for tests/test_stream.py.
//
//   stream_threads threads <level> <in1> <out1> [<in2> <out2> ...]
//       one host thread per (in, out) pair, all calling smallz4::lz4 at the same time (the reference
//       builds a fresh object per call, smallz4.h:56-64, so concurrent calls must not interfere)
//   stream_threads big <level> <base> <reps> <out> [decode]
//       one long stream through smallz4::lz4: <base> repeated <reps> times, repetition r with the
//       8 bytes at offset (r * 7919) % size replaced by r (little endian); prints the library's
//       device footprint (sz4_device_bytes of the pooled context), the stream's length and its
//       wall-clock rate (the whole smallz4::lz4 call: callbacks, PCIe both ways, kernels), after a
//       first call over one repetition that allocates the pooled context's buffers (timed apart);
//       `decode`: the frame is kept in memory instead and decoded back through sz4_unlz4_stream
//       (smallz4cat's interface), compared with the input as it arrives, and timed
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "smallz4_amd.hpp"

namespace {

std::vector<unsigned char> read_file(const char* path)
{
  std::vector<unsigned char> v;
  FILE* f = fopen(path, "rb");
  if (!f) {
    perror(path);
    exit(2);
  }
  unsigned char buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + k);
  fclose(f);
  return v;
}

struct MemIn {
  const std::vector<unsigned char>* data;
  size_t at;
};
struct FileOut {
  FILE* f;
};

size_t get_mem(void* data, size_t n, void* user)
{
  MemIn* m = static_cast<MemIn*>(user);
  const size_t k = std::min(n, m->data->size() - m->at);
  memcpy(data, m->data->data() + m->at, k);
  m->at += k;
  return k;
}

// both directions through one user pointer, as the reference's CLI does (smallz4.cpp:50-117)
struct Job {
  MemIn in;
  FILE* out;
};
size_t get_job(void* data, size_t n, void* user) { return get_mem(data, n, &static_cast<Job*>(user)->in); }
void send_job(const void* data, size_t n, void* user)
{
  if (n) fwrite(data, 1, n, static_cast<Job*>(user)->out);
}

// the long synthetic stream
struct Big {
  const std::vector<unsigned char>* base;
  uint64_t reps, pos, total;
  FILE* out;
  uint64_t sent;
  double getSecs, sendSecs;  // time spent inside the callbacks (the caller's side of the interface)
  std::vector<unsigned char>* keep = nullptr;  // the frame, kept in memory for the decode check
};
struct CallbackClock {
  double* acc;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  ~CallbackClock() { *acc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); }
};
size_t get_big(void* data, size_t n, void* user)
{
  Big* b = static_cast<Big*>(user);
  CallbackClock clock{&b->getSecs};
  unsigned char* d = static_cast<unsigned char*>(data);
  const uint64_t size = b->base->size();
  size_t k = 0;
  while (k < n && b->pos < b->total) {
    const uint64_t r = b->pos / size, o = b->pos % size;
    const uint64_t take = std::min<uint64_t>(n - k, size - o);
    memcpy(d + k, b->base->data() + o, take);
    // patch: the 8 bytes at (r * 7919) % size hold r
    const uint64_t p = (r * 7919) % size;
    for (uint64_t j = 0; j < 8; j++) {
      const uint64_t q = p + j;
      if (q >= o && q < o + take && q < size) d[k + (q - o)] = (unsigned char)(r >> (8 * j));
    }
    k += take;
    b->pos += take;
  }
  return k;
}
void send_big(const void* data, size_t n, void* user)
{
  Big* b = static_cast<Big*>(user);
  CallbackClock clock{&b->sendSecs};
  if (n && b->out) fwrite(data, 1, n, b->out);
  if (n && b->keep) b->keep->insert(b->keep->end(), (const unsigned char*)data, (const unsigned char*)data + n);
  b->sent += n;
}

// decoding the kept frame back (sz4_unlz4_stream, smallz4cat's getByte / sendBytes pattern): the output
// is compared with the regenerated stream as it arrives
struct Cat {
  const std::vector<unsigned char>* frame;
  uint64_t at;
  Big gen;       // regenerates the input stream for the comparison
  uint64_t got;  // output bytes received
  bool same;
  std::vector<unsigned char> want;
};
unsigned char cat_get(void* user)
{
  Cat* c = static_cast<Cat*>(user);
  return c->at < c->frame->size() ? (*c->frame)[c->at++] : 0;
}
void cat_send(const unsigned char* data, unsigned int n, void* user)
{
  Cat* c = static_cast<Cat*>(user);
  c->want.resize(n);
  const size_t k = get_big(c->want.data(), n, &c->gen);
  c->same = c->same && k == n && memcmp(c->want.data(), data, n) == 0;
  c->got += n;
}

}  // namespace

int main(int argc, char** argv)
{
  if (argc < 3) return 2;
  const int level = atoi(argv[2]);
  const unsigned short chain = level >= 9 ? 65535 : (unsigned short)level;
  if (std::string(argv[1]) == "threads") {
    const int n = (argc - 3) / 2;
    std::vector<std::vector<unsigned char>> inputs(n);
    std::vector<Job> jobs(n);
    for (int i = 0; i < n; i++) {
      inputs[i] = read_file(argv[3 + 2 * i]);
      jobs[i].in = MemIn{&inputs[i], 0};
      jobs[i].out = fopen(argv[4 + 2 * i], "wb");
    }
    std::vector<std::thread> threads;
    for (int i = 0; i < n; i++)
      threads.emplace_back([&, i]() { smallz4::lz4(get_job, send_job, chain, false, &jobs[i]); });
    for (auto& t : threads) t.join();
    for (auto& j : jobs) fclose(j.out);
    return 0;
  }
  if (std::string(argv[1]) == "big" && argc >= 6) {
    std::vector<unsigned char> base = read_file(argv[3]);
    // a first call of one repetition: the pooled context's device scratch and pinned host buffers are
    // allocated there (the reference builds its buffers per call too); the timed call reuses them
    Big w{&base, 1, 0, base.size(), fopen("/dev/null", "wb"), 0, 0.0, 0.0};
    const auto tw = std::chrono::steady_clock::now();
    smallz4::lz4(get_big, send_big, chain, false, &w);
    const double firstSecs = std::chrono::duration<double>(std::chrono::steady_clock::now() - tw).count();
    fclose(w.out);
    const bool decode = argc >= 7 && std::string(argv[6]) == "decode";
    std::vector<unsigned char> frame;
    Big b{&base, (uint64_t)atoll(argv[4]), 0, 0, decode ? nullptr : fopen(argv[5], "wb"), 0, 0.0, 0.0};
    if (decode) {
      frame.reserve((size_t)(b.reps * base.size() / 2 + (64 << 20)));
      b.keep = &frame;
    }
    b.total = b.reps * base.size();
    const auto t0 = std::chrono::steady_clock::now();
    smallz4::lz4(get_big, send_big, chain, false, &b);
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (b.out) fclose(b.out);
    double catSecs = 0.0;
    bool catOk = false;
    if (decode) {
      // the frame back through the decoder's stream interface (smallz4cat's unlz4_userPtr), compared
      // with the input as it arrives
      Cat cat{&frame, 0, Big{&base, b.reps, 0, b.total, nullptr, 0, 0.0, 0.0}, 0, true, {}};
      sz4_ctx* dc = NULL;
      sz4_acquire(&dc, getenv("SMALLZ4_AMD_DEVICE") ? atoi(getenv("SMALLZ4_AMD_DEVICE")) : 0);
      const auto tc = std::chrono::steady_clock::now();
      const int rc = sz4_unlz4_stream(dc, cat_get, cat_send, NULL, 0, &cat);
      catSecs = std::chrono::duration<double>(std::chrono::steady_clock::now() - tc).count();
      sz4_release(dc);
      catOk = rc == SZ4_OK && cat.same && cat.got == b.total;
    }
    // the footprint of the pooled context the call used (handed back to the pool, borrowed again)
    sz4_ctx* c = NULL;
    sz4_acquire(&c, getenv("SMALLZ4_AMD_DEVICE") ? atoi(getenv("SMALLZ4_AMD_DEVICE")) : 0);
    printf("{\"input_bytes\": %llu, \"output_bytes\": %llu, \"device_bytes\": %llu, \"seconds\": %.3f, \"MB/s\": %.1f, "
           "\"get_bytes_seconds\": %.3f, \"send_bytes_seconds\": %.3f, \"first_call_bytes\": %llu, \"first_call_seconds\": %.3f, "
           "\"decode_seconds\": %.3f, \"decode_MB/s\": %.1f, \"decode_ok\": %s}\n",
           (unsigned long long)b.total, (unsigned long long)b.sent, (unsigned long long)sz4_device_bytes(c), secs,
           b.total / secs / 1e6, b.getSecs, b.sendSecs, (unsigned long long)base.size(), firstSecs, catSecs,
           catSecs > 0 ? b.total / catSecs / 1e6 : 0.0, decode ? (catOk ? "true" : "false") : "null");
    sz4_release(c);
    return 0;
  }
  return 2;
}
