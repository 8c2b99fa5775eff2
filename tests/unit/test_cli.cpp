// CLI / daemon-loop tests: flag semantics (urfave/cli v2), precedence
// (CLI > env > config file > default, flags.go:29-40), and the run() fault
// matrix (cmd/gpu-feature-discovery/main_test.go:273-380).
#include <unistd.h>

#include <thread>

#include "cli/daemon.h"
#include "cli/flags.h"
#include "lm/node.h"
#include "resource/managers.h"
#include "sriov/sriov.h"
#include "test.h"
#include "util/dynlib.h"
#include "util/fs.h"
#include "util/log.h"
#include "util/trace.h"

using namespace gfd;
using namespace gfd::cli;

namespace {
using Env = std::map<std::string, std::string>;
Context parse(std::vector<std::string> args, Env env = {}) { return Context::parse(gfd_flags(), args, &env); }

std::string temp_dir() {
  char d[] = "/tmp/gfd-cli-XXXXXX";
  if (!mkdtemp(d)) throw std::runtime_error("mkdtemp");
  return d;
}
}  // namespace

TEST(Flags_Defaults) {
  auto c = parse({});
  EXPECT_EQ(c.String("mig-strategy"), std::string("none"));
  EXPECT_TRUE(c.Bool("fail-on-init-error"));
  EXPECT_FALSE(c.Bool("oneshot"));
  EXPECT_EQ(c.Duration("sleep-interval"), 60 * kSecond);
  EXPECT_EQ(c.String("output-file"), std::string("/etc/kubernetes/node-feature-discovery/features.d/gfd"));
  EXPECT_EQ(c.String("machine-type-file"), std::string("/sys/class/dmi/id/product_name"));
  EXPECT_FALSE(c.IsSet("oneshot"));
}

TEST(Flags_GoSyntaxVariants) {
  auto c = parse({"-oneshot", "--mig-strategy=single", "-o", "/x", "--sleep-interval", "5s", "--fail-on-init-error=false"});
  EXPECT_TRUE(c.Bool("oneshot"));
  EXPECT_EQ(c.String("mig-strategy"), std::string("single"));
  EXPECT_EQ(c.String("output-file"), std::string("/x"));
  EXPECT_EQ(c.Duration("sleep-interval"), 5 * kSecond);
  EXPECT_FALSE(c.Bool("fail-on-init-error"));
  EXPECT_TRUE(c.IsSet("output"));
  EXPECT_TRUE(c.IsSet("o"));
}

TEST(Flags_AliasesAndLastWins) {
  auto c = parse({"--output=/a", "--output-file", "/b"});
  EXPECT_EQ(c.String("o"), std::string("/b"));
}

TEST(Flags_EmptyOutputMeansStdout) {
  auto c = parse({"--output-file="});
  EXPECT_EQ(c.String("output-file"), std::string(""));
  EXPECT_TRUE(c.IsSet("output-file"));
}

TEST(Flags_BoolDoesNotConsumeNextArg) {
  auto c = parse({"--oneshot", "false"});
  EXPECT_TRUE(c.Bool("oneshot"));
  EXPECT_EQ(c.positional(), (std::vector<std::string>{"false"}));
}

TEST(Flags_StopsAtDoubleDash) {
  auto c = parse({"--", "--oneshot"});
  EXPECT_FALSE(c.Bool("oneshot"));
}

TEST(Flags_Errors) {
  EXPECT_THROW_MSG(parse({"--bogus"}), "flag provided but not defined: -bogus");
  EXPECT_THROW_MSG(parse({"--mig-strategy"}), "flag needs an argument: -mig-strategy");
  EXPECT_THROW_MSG(parse({"--oneshot=maybe"}), "invalid boolean value");
  EXPECT_THROW_MSG(parse({"--sleep-interval=10"}), "invalid value");
}

TEST(Flags_HelpAndVersion) {
  EXPECT_TRUE(parse({"-h"}).help_requested());
  EXPECT_TRUE(parse({"--version"}).version_requested());
  std::string h = help_text(gfd_flags(), "GPU Feature Discovery", "x", "v");
  EXPECT_TRUE(h.find("--output-file value, --output value, -o value") != std::string::npos);
  EXPECT_TRUE(h.find("[$GFD_MIG_STRATEGY, $MIG_STRATEGY]") != std::string::npos);
}

TEST(Flags_EnvVarsFirstPresentWins) {
  auto c = parse({}, {{"MIG_STRATEGY", "mixed"}, {"GFD_MIG_STRATEGY", "single"}});
  EXPECT_EQ(c.String("mig-strategy"), std::string("single"));
  auto c2 = parse({}, {{"MIG_STRATEGY", "mixed"}});
  EXPECT_EQ(c2.String("mig-strategy"), std::string("mixed"));
  EXPECT_TRUE(c2.IsSet("mig-strategy"));
}

TEST(Flags_CliBeatsEnv) {
  auto c = parse({"--mig-strategy=none"}, {{"GFD_MIG_STRATEGY", "single"}});
  EXPECT_EQ(c.String("mig-strategy"), std::string("none"));
}

TEST(Flags_EmptyEnvSemantics) {
  // A string env var applies even when empty; bool/duration ones are ignored.
  auto c = parse({}, {{"GFD_OUTPUT_FILE", ""}, {"GFD_ONESHOT", ""}, {"GFD_SLEEP_INTERVAL", ""}});
  EXPECT_EQ(c.String("output-file"), std::string(""));
  EXPECT_TRUE(c.IsSet("output-file"));
  EXPECT_FALSE(c.IsSet("oneshot"));
  EXPECT_FALSE(c.IsSet("sleep-interval"));
}

TEST(Flags_BadEnvValuesError) {
  EXPECT_THROW_MSG(parse({}, {{"GFD_ONESHOT", "perhaps"}}), "could not parse \"perhaps\" as bool value from environment variable \"GFD_ONESHOT\"");
  EXPECT_THROW_MSG(parse({}, {{"GFD_SLEEP_INTERVAL", "1x"}}), "as duration value");
}

TEST(LoadConfig_Precedence) {
  std::string dir = temp_dir();
  std::string file = dir + "/config.yaml";
  lm::write_file_atomically(file,
                            "version: v1\nflags:\n  migStrategy: mixed\n  failOnInitError: false\n  gfd:\n"
                            "    oneshot: true\n    sleepInterval: 10s\n",
                            0644);
  // File beats default; env beats file; CLI beats env.
  auto c = load_config(parse({"--config-file", file, "--sleep-interval=20s"}, {{"GFD_MIG_STRATEGY", "single"}}));
  EXPECT_EQ(c.mig_strategy(), std::string("single"));       // env over file
  EXPECT_FALSE(c.fail_on_init_error());                      // file over default
  EXPECT_TRUE(c.oneshot());                                  // file over default
  EXPECT_EQ(c.sleep_interval(), 20 * kSecond);               // CLI over file
  EXPECT_EQ(c.output_file(), std::string(config::kDefaultOutputFile));  // default
  fs::remove_all(dir);
}

TEST(LoadConfig_ConfigFileFromEnv) {
  std::string dir = temp_dir();
  std::string file = dir + "/c.json";
  lm::write_file_atomically(file, R"({"flags":{"migStrategy":"single"}})", 0644);
  auto c = load_config(parse({}, {{"CONFIG_FILE", file}}));
  EXPECT_EQ(c.mig_strategy(), std::string("single"));
  fs::remove_all(dir);
}

TEST(LoadConfig_BadFileErrors) {
  EXPECT_THROW_MSG(load_config(parse({"--config-file=/nonexistent/gfd.yaml"})),
                   "unable to finalize config: unable to parse config file: error opening config file");
}

// ---- run() (main_test.go) ----

namespace {
config::Config run_config(const std::string& out, const std::string& strategy, bool fail_on_init, bool oneshot) {
  config::Config c;
  c.flags.mig_strategy = strategy;
  c.flags.fail_on_init_error = fail_on_init;
  c.flags.gfd.oneshot = oneshot;
  c.flags.gfd.output_file = out;
  c.flags.gfd.sleep_interval = kSecond / 2;
  c.flags.gfd.no_timestamp = false;
  c.flags.gfd.machine_type_file = "/nonexistent/machine";
  return c;
}
}  // namespace

TEST(Run_OneshotWritesFileAndKeepsIt) {
  std::string dir = temp_dir();
  std::string out = dir + "/gfd";
  auto c = run_config(out, "none", true, true);
  resource::MockManager m({resource::new_full_gpu()});
  EXPECT_FALSE(run(m, sriov::new_mock_sriov(), c, nullptr));
  std::string data = fs::read_file(out).data;
  EXPECT_TRUE(data.find("amd.com/gpu.product=MOCKMODEL\n") != std::string::npos);
  EXPECT_TRUE(data.find("amd.com/gfd.timestamp=") != std::string::npos);
  EXPECT_TRUE(data.find("amd.com/sriov.present=true\n") != std::string::npos);
  EXPECT_EQ(m.init_calls, 1);
  EXPECT_EQ(m.shutdown_calls, 1);
  fs::remove_all(dir);
}

TEST(Run_InitErrorMatrix) {
  struct Case {
    bool error_on_init;
    bool fail_on_init;
    const char* strategy;
    bool expect_error;
  };
  const Case cases[] = {
      {true, true, "none", true},    {true, true, "bogus", true},   {true, false, "bogus", false},
      {true, false, "bogus", false}, {false, true, "none", false},  {false, true, "bogus", true},
      {false, false, "none", false}, {false, false, "bogus", true},
  };
  std::string dir = temp_dir();
  for (const auto& tc : cases) {
    auto c = run_config(dir + "/gfd", tc.strategy, tc.fail_on_init, true);
    auto mock = std::make_shared<resource::MockManager>(std::vector<resource::DevicePtr>{resource::new_full_gpu()});
    if (tc.error_on_init) mock->with_error_on_init("manager.Init error");
    auto m = resource::with_config(mock, c);
    bool threw = false;
    try {
      EXPECT_FALSE(run(*m, sriov::new_mock_sriov(), c, nullptr));
    } catch (const gfdtest::Failure&) {
      throw;
    } catch (const std::exception&) {
      threw = true;
    }
    if (threw != tc.expect_error)
      GFD_FAIL("case error_on_init=" << tc.error_on_init << " fail_on_init=" << tc.fail_on_init << " strategy="
                                     << tc.strategy << ": threw=" << threw);
  }
  fs::remove_all(dir);
}

TEST(Run_FallbackIsSticky) {
  auto mock = std::make_shared<resource::MockManager>(std::vector<resource::DevicePtr>{resource::new_full_gpu()});
  mock->with_error_on_init("boom");
  resource::FallbackManager f(mock);
  EXPECT_NO_THROW(f.Init());
  EXPECT_TRUE(f.fell_back());
  EXPECT_TRUE(f.GetDevices().empty());
  mock->init_error.reset();
  f.Init();  // still the null manager
  EXPECT_TRUE(f.GetDevices().empty());
  EXPECT_EQ(mock->init_calls, 1);
}

TEST(Run_NoTimestampOmitsLabel) {
  std::string dir = temp_dir();
  auto c = run_config(dir + "/gfd", "none", true, true);
  c.flags.gfd.no_timestamp = true;
  resource::MockManager m({resource::new_full_gpu()});
  run(m, sriov::new_mock_sriov(), c, nullptr);
  EXPECT_TRUE(fs::read_file(dir + "/gfd").data.find("gfd.timestamp") == std::string::npos);
  fs::remove_all(dir);
}

TEST(Run_NullManagerWritesOnlyTimestampAndSriov) {
  std::string dir = temp_dir();
  auto c = run_config(dir + "/gfd", "none", true, true);
  resource::NullManager m;
  run(m, sriov::new_empty_sriov(), c, nullptr);
  std::string data = fs::read_file(dir + "/gfd").data;
  EXPECT_TRUE(data.find("amd.com/gfd.timestamp=") == 0);
  EXPECT_EQ(std::count(data.begin(), data.end(), '\n'), 1L);
  fs::remove_all(dir);
}

TEST(LabelCycle_RecordsPhases) {
  for (bool oneshot : {true, false}) {
    auto c = run_config("", "none", true, oneshot);
    resource::MockManager m({resource::new_full_gpu()});
    auto ts = lm::NewTimestampLabeler(c, 1);
    auto r = label_cycle(m, sriov::new_empty_sriov(), c, ts, false);
    std::vector<std::string> names;
    int machine = 0;  // where depends on which thread read the facts
    for (const auto& p : r.phases) {
      if (p.first == "facts.machine") {
        ++machine;
        continue;
      }
      if (p.first == "sriov.self") continue;  // this thread took the SR-IOV lookup over
      names.push_back(p.first);
    }
    EXPECT_EQ(machine, 1);
    if (oneshot) {
      // A Job reads the node facts and does the lookup on this thread.
      EXPECT_EQ(names, (std::vector<std::string>{"placement", "versions", "init", "enumerate", "label", "shutdown",
                                                 "sriov", "facts", "merge"}));
    } else {
      EXPECT_EQ(names, (std::vector<std::string>{"placement", "versions", "submit", "init", "enumerate", "facts.wait",
                                                 "label", "shutdown", "sriov.join", "facts.start", "facts(overlapped)",
                                                 "sriov(overlapped)", "merge"}));
    }
    // Every top-level phase is named: what is left is bookkeeping.
    EXPECT_TRUE(r.other_ns >= 0 && r.other_ns < r.total_ns);
    EXPECT_TRUE(r.total_ns > 0);
    EXPECT_EQ(r.labels["amd.com/gfd.timestamp"], std::string("1"));
  }
}

namespace {
// An SR-IOV source that records a detail, as BoundAmdPCI does.
struct RecordingSriov : sriov::Interface {
  std::vector<sriov::Function> Devices() override {
    trace::record("pci.test", 5000);
    return {};
  }
};
}  // namespace

TEST(LabelCycle_UntracedRecordsNothingAndLabelsTheSame) {
  // The daemon without --trace-timing: no phase anywhere (the SR-IOV
  // source's own record included, on whichever thread it ran), the same
  // labels, and a traced cycle afterwards records as before.
  for (bool oneshot : {true, false}) {
    auto c = run_config("", "none", true, oneshot);
    resource::MockManager m({resource::new_full_gpu()});
    auto ts = lm::NewTimestampLabeler(c, 1);
    for (int i = 0; i < 10; ++i) {
      auto quiet = label_cycle(m, std::make_shared<RecordingSriov>(), c, ts, false, false);
      EXPECT_TRUE(quiet.phases.empty());
      EXPECT_EQ(quiet.other_ns, quiet.total_ns);
      auto traced = label_cycle(m, std::make_shared<RecordingSriov>(), c, ts, false, true);
      EXPECT_TRUE(quiet.labels == traced.labels);
      int n = 0;
      for (const auto& p : traced.phases) n += p.first == "pci.test";
      EXPECT_EQ(n, 1);
    }
  }
}

TEST(Trace_UntracedSpansAndStampsReadNoClock) {
  trace::begin_cycle(false);
  EXPECT_FALSE(trace::active());
  EXPECT_EQ(trace::stamp(), 0);
  { trace::Span s("write"); }
  trace::record_since("write.rename", trace::stamp());
  std::thread worker([] {
    trace::Capture c(false);  // an untraced cycle's task
    EXPECT_FALSE(trace::active());
    trace::record("pci.x", 1);
    EXPECT_TRUE(c.take().empty());
  });
  worker.join();
  EXPECT_TRUE(trace::phases().empty());
  EXPECT_EQ(trace::top_level_ns(), 0);
  trace::begin_cycle(true);
  { trace::Span s("write"); }
  EXPECT_EQ(trace::phases().size(), static_cast<size_t>(1));
}

TEST(Trace_CaptureHandsAWorkersRecordsToTheCycleOnce) {
  trace::begin_cycle();
  std::vector<trace::Phase> got;
  std::thread worker([&] {
    trace::record("dropped", 1);  // a worker records nothing of its own
    trace::Capture c;
    { trace::Span s("pci.x"); }
    trace::record("pci.y", 2);
    got = c.take();
  });
  worker.join();
  EXPECT_EQ(got.size(), static_cast<size_t>(2));
  EXPECT_EQ(got[0].first, std::string("pci.x"));
  EXPECT_EQ(got[1].first, std::string("pci.y"));
  {
    // On the cycle thread the records are already the cycle's.
    trace::Capture c;
    trace::record("pci.z", 3);
    EXPECT_TRUE(c.take().empty());
  }
  EXPECT_EQ(trace::phases().size(), static_cast<size_t>(1));
  EXPECT_EQ(trace::phases()[0].first, std::string("pci.z"));
}

TEST(LabelCycle_RecordsTheSriovLookupsDetailOnceWhereverItRan) {
  auto c = run_config("", "none", true, true);
  resource::MockManager m({resource::new_full_gpu()});
  auto ts = lm::NewTimestampLabeler(c, 1);
  for (int i = 0; i < 20; ++i) {
    auto r = label_cycle(m, std::make_shared<RecordingSriov>(), c, ts, false);
    int n = 0;
    for (const auto& p : r.phases) n += p.first == "pci.test";
    EXPECT_EQ(n, 1);
  }
}

namespace {
// Runs fn with stderr redirected to a temporary file; returns what it wrote
// so far each time `peek` is called, and everything at the end.
struct StderrCapture {
  char path[32] = "/tmp/gfd-stderr-XXXXXX";
  int fd = -1, saved = -1;
  StderrCapture() {
    fd = mkstemp(path);
    fflush(stderr);
    saved = dup(2);
    dup2(fd, 2);
  }
  std::string peek() {
    fflush(stderr);
    return fs::read_file(path).data;
  }
  ~StderrCapture() {
    fflush(stderr);
    dup2(saved, 2);
    close(saved);
    close(fd);
    unlink(path);
  }
};
}  // namespace

TEST(LogHold_WritesTheCycleLinesTogetherInOrder) {
  bool was = log::set_quiet(false);
  std::string held, after, nested;
  {
    StderrCapture cap;
    {
      log::Hold hold;
      log::printf("Writing labels to output file");
      log::printf("Sleeping for %s", "60s");
      held = cap.peek();  // nothing yet
      hold.flush();
      after = cap.peek();
      {
        log::Hold inner;  // nested: the outer one writes
        log::printf("inner");
      }
      nested = cap.peek();
    }
    nested = cap.peek();
  }
  log::set_quiet(was);
  EXPECT_EQ(held, std::string(""));
  auto a = after.find("Writing labels to output file"), b = after.find("Sleeping for 60s");
  EXPECT_TRUE(a != std::string::npos && b != std::string::npos && a < b);
  EXPECT_TRUE(nested.find("inner") != std::string::npos);
}

TEST(Log_LinesLongerThanTheBufferAreWrittenWhole) {
  // The config dump and a backend disagreement's two device lists can run
  // past the 4 KiB stack buffer.
  bool was = log::set_quiet(false);
  std::string big(10000, 'x'), out;
  {
    StderrCapture cap;
    log::printf("Running with config: %s|end", big.c_str());
    out = cap.peek();
  }
  log::set_quiet(was);
  EXPECT_TRUE(out.find("Running with config: " + big + "|end\n") != std::string::npos);
}

TEST(DynLib_ReportsWhyNoCandidateLoaded) {
  DynLib lib;
  EXPECT_FALSE(lib.open({"/nonexistent/libnothing.so", "libgfd-no-such-library.so.9"}));
  EXPECT_TRUE(lib.last_error().find("libgfd-no-such-library.so.9") != std::string::npos);
  EXPECT_TRUE(lib.symbol("anything") == nullptr);
  EXPECT_TRUE(lib.open({"libc.so.6"}));
  EXPECT_EQ(lib.path(), std::string("libc.so.6"));
  int (*getpid_fn)() = nullptr;
  EXPECT_TRUE(lib.bind("getpid", getpid_fn) && getpid_fn() == ::getpid());
  lib.close();
  EXPECT_TRUE(lib.symbol("getpid") == nullptr);
}

TEST(LogHold_NestedHoldsWriteAWarningAfterEverythingHeldBefore) {
  // The outer Hold's earlier lines go out before the inner Hold's, and both
  // before the warning; short messages ("Warn", "Err") are never compared
  // past their end.
  bool was = log::set_quiet(false);
  std::string at_warning, at_end;
  {
    StderrCapture cap;
    {
      log::Hold outer;
      log::printf("outer-1");
      {
        log::Hold inner;
        log::printf("inner-1");
        log::printf("Warn");
        log::printf("Err");
        EXPECT_EQ(cap.peek(), std::string(""));
        log::printf("Warning: w");
        at_warning = cap.peek();
        log::printf("inner-2");
      }
      log::printf("outer-2");
    }
    at_end = cap.peek();
  }
  log::set_quiet(was);
  auto o1 = at_warning.find("outer-1"), i1 = at_warning.find("inner-1"), wn = at_warning.find("Warn\n"),
       er = at_warning.find("Err\n"), w = at_warning.find("Warning: w");
  EXPECT_TRUE(o1 != std::string::npos && i1 != std::string::npos && w != std::string::npos);
  EXPECT_TRUE(o1 < i1 && i1 < wn && wn < er && er < w);
  auto i2 = at_end.find("inner-2"), o2 = at_end.find("outer-2");
  EXPECT_TRUE(w < i2 && i2 < o2 && o2 != std::string::npos);
  EXPECT_EQ(at_end.find("outer-1", o1 + 1), std::string::npos);  // written once
}

TEST(LogHold_WritesWarningsAtOnceWithWhatCameBefore) {
  // A cycle that hangs after a warning (a wedged library call) or is killed
  // must already have said why: warnings and errors are not held.
  bool was = log::set_quiet(false);
  std::string before, at_warning, at_error;
  {
    StderrCapture cap;
    log::Hold hold;
    log::printf("Writing labels to output file");
    before = cap.peek();
    log::printf("Warning: resource manager shutdown failed: %s", "x");
    at_warning = cap.peek();
    log::printf("routine");
    log::printf("Error: %s", "y");
    at_error = cap.peek();
  }
  log::set_quiet(was);
  EXPECT_EQ(before, std::string(""));
  auto a = at_warning.find("Writing labels"), b = at_warning.find("Warning: resource manager");
  EXPECT_TRUE(a != std::string::npos && b != std::string::npos && a < b);
  auto c = at_error.find("routine"), d = at_error.find("Error: y");
  EXPECT_TRUE(c != std::string::npos && d != std::string::npos && b < c && c < d);
}
