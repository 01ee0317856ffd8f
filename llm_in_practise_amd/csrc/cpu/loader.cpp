// Token-block data loader (the reference's ``TokenizedDataset`` + ``DataLoader`` +
// ``DistributedSampler`` role: ``ddp_gpt_wikitext2.py:56-81,242-257``) as a native producer.
//
// A flat int64 token stream is cut into blocks of (block_size + 1) tokens; each epoch the
// block order is shuffled with a seeded mt19937_64 (same permutation on every rank), ranks
// take a strided shard (DistributedSampler semantics, drop_last), and a background thread
// assembles [batch, block_size] input / target pairs into a ring of pinned host buffers so
// the H2D copy (non_blocking) overlaps compute.  Resume is exact: (epoch, cursor) restore
// the position.
#include <torch/extension.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <numeric>
#include <random>
#include <thread>
#include <vector>

namespace {

class TokenBlockLoader {
 public:
  TokenBlockLoader(torch::Tensor tokens, int64_t block_size, int64_t batch, int64_t rank, int64_t world, uint64_t seed,
                   bool shuffle, int64_t prefetch, bool pin)
      : tokens_(tokens.to(torch::kLong).contiguous()),
        block_(block_size),
        batch_(batch),
        rank_(rank),
        world_(world),
        seed_(seed),
        shuffle_(shuffle),
        prefetch_(std::max<int64_t>(1, prefetch)),
        pin_(pin) {
    TORCH_CHECK(block_ > 0 && batch_ > 0 && world_ > 0 && rank_ >= 0 && rank_ < world_, "bad loader args");
    nblocks_ = tokens_.numel() / (block_ + 1);
    per_rank_ = nblocks_ / world_;
    steps_per_epoch_ = per_rank_ / batch_;
    TORCH_CHECK(steps_per_epoch_ > 0, "dataset too small for batch*world");
    start_epoch(0, 0);
  }
  ~TokenBlockLoader() { stop(); }

  int64_t steps_per_epoch() const { return steps_per_epoch_; }
  int64_t num_blocks() const { return nblocks_; }
  std::pair<int64_t, int64_t> position() const { return {epoch_, cursor_}; }

  // set position (resume) and restart the producer
  void start_epoch(int64_t epoch, int64_t cursor) {
    stop();
    epoch_ = epoch;
    cursor_ = cursor;
    produced_ = cursor;
    build_order(epoch);
    running_ = true;
    worker_ = std::thread([this] { this->run(); });
  }

  // next (inputs, targets) for this rank; advances epochs automatically
  std::vector<torch::Tensor> next() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return !queue_.empty(); });
    auto item = queue_.front();
    queue_.pop_front();
    cv_.notify_all();
    lk.unlock();
    cursor_ = item.cursor + 1;
    epoch_ = item.epoch;
    if (cursor_ >= steps_per_epoch_) {
      epoch_ += 1;
      cursor_ = 0;
    }
    return {item.x, item.y};
  }

 private:
  struct Item {
    torch::Tensor x, y;
    int64_t epoch, cursor;
  };

  void build_order(int64_t ep) {
    order_.resize(nblocks_);
    std::iota(order_.begin(), order_.end(), 0);
    if (shuffle_) {
      std::mt19937_64 rng(seed_ + (uint64_t)ep * 0x9E3779B97F4A7C15ull);
      std::shuffle(order_.begin(), order_.end(), rng);
    }
  }

  void run() {
    const int64_t* src = tokens_.data_ptr<int64_t>();
    int64_t ep = epoch_, cur = produced_;
    while (running_) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return !running_ || (int64_t)queue_.size() < prefetch_; });
        if (!running_) return;
      }
      auto opts = torch::TensorOptions().dtype(torch::kLong).pinned_memory(pin_);
      torch::Tensor x = torch::empty({batch_, block_}, opts), y = torch::empty({batch_, block_}, opts);
      int64_t* X = x.data_ptr<int64_t>();
      int64_t* Y = y.data_ptr<int64_t>();
      for (int64_t b = 0; b < batch_; ++b) {
        // DistributedSampler: rank r takes indices r, r+world, ... of the shuffled order
        const int64_t local = cur * batch_ + b;
        const int64_t blk = order_[local * world_ + rank_];
        const int64_t* s = src + blk * (block_ + 1);
        std::memcpy(X + b * block_, s, sizeof(int64_t) * block_);
        std::memcpy(Y + b * block_, s + 1, sizeof(int64_t) * block_);
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        queue_.push_back({x, y, ep, cur});
      }
      cv_.notify_all();
      if (++cur >= steps_per_epoch_) {
        cur = 0;
        ++ep;
        build_order(ep);  // producer-private: the consumer only sees finished Items
      }
    }
  }

  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      running_ = false;
    }
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
    queue_.clear();
  }

  torch::Tensor tokens_;
  int64_t block_, batch_, rank_, world_;
  uint64_t seed_;
  bool shuffle_;
  int64_t prefetch_;
  bool pin_;
  int64_t nblocks_ = 0, per_rank_ = 0, steps_per_epoch_ = 0;
  int64_t epoch_ = 0, cursor_ = 0, produced_ = 0;
  std::vector<int64_t> order_;
  std::deque<Item> queue_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<bool> running_{false};
  std::thread worker_;
};

}  // namespace

#ifndef LIPA_SANITIZER_HARNESS
void register_loader(pybind11::module& m) {
  pybind11::class_<TokenBlockLoader>(m, "TokenBlockLoader")
      .def(pybind11::init<torch::Tensor, int64_t, int64_t, int64_t, int64_t, uint64_t, bool, int64_t, bool>(),
           pybind11::arg("tokens"), pybind11::arg("block_size"), pybind11::arg("batch"), pybind11::arg("rank") = 0,
           pybind11::arg("world") = 1, pybind11::arg("seed") = 42, pybind11::arg("shuffle") = true,
           pybind11::arg("prefetch") = 4, pybind11::arg("pin") = false)
      .def("next", &TokenBlockLoader::next, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("start_epoch", &TokenBlockLoader::start_epoch)
      .def("position", &TokenBlockLoader::position)
      .def_property_readonly("steps_per_epoch", &TokenBlockLoader::steps_per_epoch)
      .def_property_readonly("num_blocks", &TokenBlockLoader::num_blocks);
}
#endif  // LIPA_SANITIZER_HARNESS
