// Concurrency stress driver for the native controller engine, built with
// ThreadSanitizer or AddressSanitizer+UBSan by tests/test_sanitizers.py
// (the reference has no sanitizer configs and several latent
// races on metadata_ / community_evaluations_ / learners_, controller.cc:
// 473, 515, 673-683; this engine serialises its state behind one mutex and
// this driver is the evidence).
//
// Usage: engine_stress <input dir> <threads> <iterations>
// The input dir holds serialized protos written by the test:
//   params_sync.bin params_async.bin model.bin entity_<i>.bin dataset_<i>.bin
//   completed_<i>.bin
// Learner threads join, complete tasks and leave/rejoin concurrently with a
// reader thread that hammers every lineage / metadata query and a failure
// detector thread that evicts learners.  Expected engine errors
// (StatusError: stale token, evicted learner, ...) are counted, not fatal.
#include <atomic>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "engine/controller.h"

static std::string slurp(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) {
    std::fprintf(stderr, "missing %s\n", p.c_str());
    std::exit(2);
  }
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

static int run(const std::string& dir, const std::string& params, int nthreads, int iters) {
  mfl::Controller ctrl(slurp(dir + "/" + params));
  ctrl.replace_community_model(slurp(dir + "/model.bin"));
  std::atomic<long> ok{0}, expected_errors{0};
  std::atomic<bool> done{false};
  std::vector<std::thread> ts;
  for (int i = 0; i < nthreads; ++i) {
    ts.emplace_back([&, i] {
      const std::string se = slurp(dir + "/entity_" + std::to_string(i) + ".bin");
      const std::string ds = slurp(dir + "/dataset_" + std::to_string(i) + ".bin");
      const std::string task = slurp(dir + "/completed_" + std::to_string(i) + ".bin");
      std::string id, tok;
      auto join = [&] {
        mfl::Dispatch d;
        auto r = ctrl.add_learner(se, ds, &d);
        id = r.first;
        tok = r.second;
      };
      join();
      for (int k = 0; k < iters; ++k) {
        try {
          auto d = ctrl.learner_completed_task(id, tok, task);
          ok += 1 + (long)d.run_tasks.size();
        } catch (const mfl::StatusError&) {
          ++expected_errors;  // evicted by the detector thread: rejoin
          try {
            join();
          } catch (const mfl::StatusError&) {
            ++expected_errors;
          }
        }
        if (k % 17 == 16) {  // leave and rejoin
          try {
            ctrl.remove_learner(id, tok);
            join();
          } catch (const mfl::StatusError&) {
            ++expected_errors;
          }
        }
      }
    });
  }
  std::thread reader([&] {
    while (!done) {
      (void)ctrl.runtime_metadata_lineage(-1);
      (void)ctrl.community_evaluation_lineage(-1);
      (void)ctrl.participating_learners();
      (void)ctrl.community_model();
      (void)ctrl.community_model_lineage(2);
      (void)ctrl.local_task_lineage(-1, ctrl.learner_ids());
      (void)ctrl.global_iteration();
      ++ok;
    }
  });
  std::thread detector([&] {
    int n = 0;
    while (!done) {
      auto ids = ctrl.learner_ids();
      if (!ids.empty() && (++n % 7) == 0) {
        try {
          (void)ctrl.evict_learner(ids[n % ids.size()]);
        } catch (const mfl::StatusError&) {
          ++expected_errors;
        }
      }
      std::this_thread::yield();
    }
  });
  for (auto& t : ts) t.join();
  done = true;
  reader.join();
  detector.join();
  std::printf("%s: ok=%ld expected_errors=%ld global_iteration=%u learners=%zu evicted=%u\n",
              params.c_str(), ok.load(), expected_errors.load(), ctrl.global_iteration(),
              ctrl.num_learners(), ctrl.evicted());
  return ctrl.global_iteration() > 0 ? 0 : 3;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <dir> <threads> <iterations>\n", argv[0]);
    return 2;
  }
  const int nt = std::atoi(argv[2]), it = std::atoi(argv[3]);
  int rc = run(argv[1], "params_sync.bin", nt, it);
  if (rc) return rc;
  return run(argv[1], "params_async.bin", nt, it);
}
