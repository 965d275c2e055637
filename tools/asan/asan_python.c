/* The Python interpreter as an executable linked with the sanitizer runtimes (tools/asan/Makefile):
 * ASan must be the first runtime in the process, which a plain `python3` plus a sanitized
 * shared library loaded by ctypes does not give. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

int main(int argc, char** argv) { return Py_BytesMain(argc, argv); }
