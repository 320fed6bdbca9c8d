// CIFAR binary-format reader (native replacement for torchvision.datasets.CIFAR100 used by
// the reference, src/workers/worker.py:158-164). Reads the official *binary* distribution
// (cifar-100-binary/{train,test}.bin: per record 1 coarse-label byte, 1 fine-label byte,
// 3072 bytes planar RGB; cifar-10-batches-bin: 1 label byte + 3072 bytes) and converts it to
// the NHWC uint8 layout the device augmentation kernel consumes. A thread pool converts
// chunks in parallel. No pickle is ever involved.
#include <cstdint>
#include <cstdio>
#include <thread>
#include <vector>

extern "C" {

// Returns the number of records in the file (or -1), given the label byte count per record.
long psx_cifar_count(const char* path, int label_bytes) {
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  fseek(f, 0, SEEK_END);
  const long sz = ftell(f);
  fclose(f);
  const long rec = label_bytes + 3072;
  if (sz % rec) return -1;
  return sz / rec;
}

// label_index: which label byte to keep (CIFAR-100: 1 = fine label). out_img: [n][32][32][3].
long psx_cifar_read(const char* path, int label_bytes, int label_index, uint8_t* out_img, int32_t* out_labels,
                    long max_records, int threads) {
  const long n_all = psx_cifar_count(path, label_bytes);
  if (n_all < 0) return -1;
  const long n = (max_records > 0 && max_records < n_all) ? max_records : n_all;
  const long rec = label_bytes + 3072;
  std::vector<uint8_t> raw((size_t)n * rec);
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  const size_t got = fread(raw.data(), 1, raw.size(), f);
  fclose(f);
  if (got != raw.size()) return -1;
  if (threads < 1) threads = 1;
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) {
    pool.emplace_back([&, t]() {
      for (long i = t; i < n; i += threads) {
        const uint8_t* r = raw.data() + (size_t)i * rec;
        out_labels[i] = r[label_index];
        const uint8_t* px = r + label_bytes;
        uint8_t* o = out_img + (size_t)i * 3072;
        for (int p = 0; p < 1024; ++p) {
          o[p * 3 + 0] = px[p];
          o[p * 3 + 1] = px[1024 + p];
          o[p * 3 + 2] = px[2048 + p];
        }
      }
    });
  }
  for (auto& th : pool) th.join();
  return n;
}

}  // extern "C"
