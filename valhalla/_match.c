/* valhalla._match: SegmentMatcher.Match in one CPython call (round 6).
 *
 * The reference's service calls Match once per /report request from its worker threads
 * (py/reporter_service.py:240).  Through ctypes each call costs two foreign calls (rm_match,
 * rm_free), a c_void_p, byref, string_at and a decode, all while holding the GIL; with 64
 * threads the GIL-serialised part of a 60-point request was ~15 us.  Here the whole call is one
 * C function: the request's bytes go to rm_match with the GIL released, the reply is decoded
 * straight from the library's buffer and freed.  Same contract as the ctypes path: str or bytes
 * in, str out, RuntimeError with rm_last_error()'s message on failure.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <stdint.h>
#include <string.h>

#include "../include/reporter_match.h"

static PyObject* py_match(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 2) {
    PyErr_SetString(PyExc_TypeError, "match(handle, trace_json)");
    return NULL;
  }
  const unsigned long long h = PyLong_AsUnsignedLongLong(args[0]);
  if (PyErr_Occurred()) return NULL;
  if (h == 0) {
    PyErr_SetString(PyExc_RuntimeError, "matcher is NULL");   /* the library's own message */
    return NULL;
  }
  PyObject* obj = args[1];
  const char* s;
  if (PyBytes_Check(obj)) {
    s = PyBytes_AS_STRING(obj);
  } else if (PyUnicode_Check(obj)) {
    s = PyUnicode_AsUTF8(obj);   /* cached in the str object, which the caller keeps alive */
    if (!s) return NULL;
  } else {
    PyErr_SetString(PyExc_TypeError, "trace_json must be str or bytes");
    return NULL;
  }
  char* out = NULL;
  int rc;
  Py_INCREF(obj);   /* its buffer is read without the GIL */
  Py_BEGIN_ALLOW_THREADS
  rc = rm_match((rm_matcher*)(uintptr_t)h, s, &out);
  Py_END_ALLOW_THREADS
  Py_DECREF(obj);
  if (rc != 0) {
    PyErr_SetString(PyExc_RuntimeError, rm_last_error());
    return NULL;
  }
  PyObject* r = PyUnicode_DecodeUTF8(out, (Py_ssize_t)strlen(out), "strict");
  rm_free(out);
  return r;
}

static PyMethodDef kMethods[] = {
    {"match", (PyCFunction)(void (*)(void))py_match, METH_FASTCALL,
     "match(handle, trace_json) -> str: rm_match on an rm_matcher handle, GIL released"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_match",
                                     "SegmentMatcher.Match without ctypes (libreporter_match.so)", -1, kMethods,
                                     NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__match(void) { return PyModule_Create(&kModule); }
