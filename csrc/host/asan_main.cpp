// Host AddressSanitizer harness for the native runtime.
//
// The engine (csrc/engine.cpp) and the host side of every kernel file are compiled with
// `-Xarch_host -fsanitize=address` (device code unchanged) into THIS executable, which embeds
// the Python interpreter and registers the engine as the built-in module `_dlap_hip` (engine.cpp
// built with -DDLAP_EMBED). The ASan runtime is linked into the executable, so it is first in
// the process without any preloading, and every host allocation of the runtime, the launchers
// and the pybind11 bindings is checked. Usage:
//     dlap_asan_python SCRIPT.py [args...]       (runs SCRIPT as __main__)
//     dlap_asan_python -c CODE [args...]         (python -c; multiprocessing's spawned children
//                                                  re-run sys.executable this way)
#include <pybind11/embed.h>

#include <cstdio>
#include <string>

namespace py = pybind11;

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s SCRIPT.py [args...]\n", argv[0]);
    return 2;
  }
  py::scoped_interpreter guard{};
  int rc = 0;
  try {
    py::module_ sys = py::module_::import("sys");
    const bool code = std::string(argv[1]) == "-c" && argc >= 3;
    py::list av;
    if (code) av.append("-c");
    for (int i = code ? 3 : 1; i < argc; ++i) av.append(argv[i]);
    sys.attr("argv") = av;
    // the package's loader finds the instrumented engine under its usual module name
    py::module_ eng = py::module_::import("_dlap_hip");
    sys.attr("modules")["deeplearninginassetpricing_paperreplication_amd._dlap_hip"] = eng;
    if (code) py::exec(argv[2], py::module_::import("__main__").attr("__dict__"));
    else py::module_::import("runpy").attr("run_path")(argv[1], py::arg("run_name") = "__main__");
  } catch (py::error_already_set& e) {
    if (e.matches(PyExc_SystemExit)) {
      py::object code = e.value().attr("code");
      rc = code.is_none() ? 0 : (py::isinstance<py::int_>(code) ? code.cast<int>() : 1);
    } else {
      std::fprintf(stderr, "%s\n", e.what());
      rc = 1;
    }
  }
  return rc;
}
