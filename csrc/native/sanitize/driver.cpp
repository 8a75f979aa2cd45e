// Host-sanitizer driver for the native index builders.
//
// The `_native` pybind11 module is linked STATICALLY into this executable,
// which is built with -fsanitize=address,undefined, and registered as a
// built-in module before an embedded CPython starts.  ASan is then the first
// runtime in the process (no LD_PRELOAD needed), so every heap access the
// builders make on numpy-owned and self-owned buffers is checked.  The
// embedded interpreter runs a fuzz script (tools/sanitize/fuzz_native.py)
// that drives all entry points with random and edge-case corpora and checks
// them against Python oracles.
#include <Python.h>

#include <cstdio>

extern "C" PyObject* PyInit__native();

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <script.py> [args]\n", argv[0]);
    return 2;
  }
  if (PyImport_AppendInittab("_native", &PyInit__native) != 0) return 3;
  Py_Initialize();
  wchar_t** wargv = static_cast<wchar_t**>(PyMem_RawMalloc(sizeof(wchar_t*) * (argc - 1)));
  for (int i = 1; i < argc; ++i) wargv[i - 1] = Py_DecodeLocale(argv[i], nullptr);
  PySys_SetArgvEx(argc - 1, wargv, 0);
  FILE* f = std::fopen(argv[1], "r");
  if (!f) {
    std::perror(argv[1]);
    return 4;
  }
  const int rc = PyRun_SimpleFileEx(f, argv[1], 1);
  const int fin = Py_FinalizeEx();
  for (int i = 0; i < argc - 1; ++i) PyMem_RawFree(wargv[i]);
  PyMem_RawFree(wargv);
  return (rc == 0 && fin == 0) ? 0 : 1;
}
