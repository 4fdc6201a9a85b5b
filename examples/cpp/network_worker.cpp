// Native pipeline stage worker: one process per stage, driven over TCP by a pipeline coordinator
// (dcnn_amd.parallel.pipeline.DistributedCoordinator, or examples/sync_pipeline_coordinator.py).
//
//   dcnn_amd/bin/network_worker <port> [--host 0.0.0.0] [--verbose]
//
// Listens on <port>, waits for CONFIG_TRANSFER (the stage's partition, optimizer, device and
// neighbours as the StageConfig JSON), dials the next stage, and runs the stage event loop
// (forward / backward jobs, parameter updates, parameter and optimizer-state transfer,
// checkpoints, status, load reports, heartbeats) until SHUTDOWN. The partition runs on the C++
// host API: CPU (fp32) or GPU (the routed MFMA kernels), as the configuration says.
// Reference parity: examples/network_worker.cpp:14-194, include/pipeline/network_stage_worker.hpp:25-114.
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#include "../../dcnn_amd/csrc/native/comm.h"  // (Communicator interface)
#include "dcnn/pipeline.hpp"

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: network_worker <port> [--host H] [--verbose]\n");
    return 2;
  }
  const int port = std::atoi(argv[1]);
  std::string host = "0.0.0.0";
  bool verbose = false;
  for (int i = 2; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--host" && i + 1 < argc) host = argv[++i];
    else if (a == "--verbose") verbose = true;
  }
  try {
    int bound = 0;
    auto comm = dcnn::make_tcp_communicator("worker@" + std::to_string(port), host, port, &bound);
    dcnn::PipelineStage stage(comm.get(), verbose);
    std::printf("native stage worker listening on port %d (pid %d)\n", bound, (int)getpid());
    std::fflush(stdout);
    stage.run();
    comm->close();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "network_worker: %s\n", e.what());
    return 1;
  }
  return 0;
}
