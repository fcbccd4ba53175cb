// Standalone controller executable (reference: metisfl/controller/
// controller_main.cc:31-99, which hard-codes a FedAvg / synchronous
// controller on port 50051 and serves until SIGINT).
//
// The engine (scheduler, aggregation incl. the GPU backend, model store,
// CKKS) is native; the gRPC server is grpcio's (no C++ gRPC library exists in
// this image).  This binary embeds the CPython interpreter, so it starts like
// the reference's: `build/native/metisfl_controller [--port N]
// [--checkpoint_dir DIR] [-e HEX -g HEX -c HEX -m HEX -s HEX]` -- the hex
// arguments are the serialized protos of `python -m metisfl_amd.controller`,
// the defaults the reference's (FedAvg + NUM_TRAINING_EXAMPLES, synchronous,
// in-memory store).  SIGINT / SIGTERM shut the servicer down.
#include <pybind11/embed.h>

#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

namespace py = pybind11;

int main(int argc, char** argv) {
  std::vector<std::string> args;
  std::string port;
  for (int i = 1; i < argc; ++i) {
    if (std::strcmp(argv[i], "--port") == 0 && i + 1 < argc) {
      port = argv[++i];
      continue;
    }
    if (std::strcmp(argv[i], "-h") == 0 || std::strcmp(argv[i], "--help") == 0) {
      std::cout << "usage: metisfl_controller [--port N] [--checkpoint_dir DIR] "
                   "[-e|-g|-c|-m|-s HEX_SERIALIZED_PROTO]\n";
      return 0;
    }
    args.emplace_back(argv[i]);
  }
  py::scoped_interpreter interp;
  try {
    py::module_ sys = py::module_::import("sys");
    // the package root: METISFL_AMD_ROOT, else two levels above build/native/
    const char* root = std::getenv("METISFL_AMD_ROOT");
    std::string r = root ? root : std::string(METISFL_AMD_DEFAULT_ROOT);
    sys.attr("path").attr("insert")(0, r);
    py::module_ cli = py::module_::import("metisfl_amd.controller.__main__");
    if (!port.empty()) {
      py::object ent = py::module_::import("metisfl_amd.utils.proto_messages_factory")
                           .attr("MetisProtoMessages")
                           .attr("construct_server_entity_pb")("[::]", std::stoi(port));
      std::string hex = py::bytes(ent.attr("SerializeToString")()).attr("hex")().cast<std::string>();
      args.insert(args.begin(), {"-e", hex});
    }
    py::list pyargs;
    for (auto& a : args) pyargs.append(a);
    cli.attr("main")(pyargs);
  } catch (py::error_already_set& e) {
    std::cerr << "metisfl_controller: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
