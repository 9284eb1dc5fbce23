/* mgn_pycall.c -- a CPython binding of mgn_rollout for the per-launch host path.
 *
 * BatchedEnv.rollout_launcher's loop is one call per K-step launch.  Through
 * ctypes that call costs ~3.5 us of argument conversion and libffi dispatch
 * (DESIGN.md §5), comparable to a tenth of a 20-step launch.  This module is
 * linked against libmadigan_hip.so and calls its mgn_rollout entry point
 * (include/madigan_amd.h) with the arguments unpacked by METH_FASTCALL, the
 * way the reference's pybind11 Env.step binding calls Env::step.
 *
 *   rollout(env, actions, k, traj) -> int   (= mgn_rollout(env, actions, k, traj))
 *   synchronize_spin(env) -> int            (= mgn_synchronize_spin(env): polling)
 *   synchronize(env) -> int                 (= mgn_synchronize(env): the handle's
 *                                            stream, not the whole device)
 *
 * env is the handle mgn_create returned, actions the (K, N, A) int8 device
 * actions, traj the mgn_traj the launcher validated -- the values the ctypes
 * call passes.  Plain host C; no torch types, no GPU code.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

#include "madigan_amd.h"

static PyObject *rollout(PyObject *self, PyObject *const *args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 4) {
    PyErr_SetString(PyExc_TypeError, "rollout(env, actions, k, traj) takes 4 integer arguments");
    return NULL;
  }
  mgn_env *env = (mgn_env *)PyLong_AsVoidPtr(args[0]);
  const int8_t *actions = (const int8_t *)PyLong_AsVoidPtr(args[1]);
  const long k = PyLong_AsLong(args[2]);
  const mgn_traj *traj = (const mgn_traj *)PyLong_AsVoidPtr(args[3]);
  if (PyErr_Occurred()) return NULL;
  if (env == NULL || traj == NULL) {
    PyErr_SetString(PyExc_ValueError, "rollout: null handle or trajectory");
    return NULL;
  }
  return PyLong_FromLong(mgn_rollout(env, actions, (int32_t)k, traj));
}

static PyObject *synchronize(PyObject *self, PyObject *arg) {
  (void)self;
  mgn_env *env = (mgn_env *)PyLong_AsVoidPtr(arg);
  if (PyErr_Occurred()) return NULL;
  if (env == NULL) {
    PyErr_SetString(PyExc_ValueError, "synchronize: null handle");
    return NULL;
  }
  int rc;
  Py_BEGIN_ALLOW_THREADS rc = mgn_synchronize(env);
  Py_END_ALLOW_THREADS return PyLong_FromLong(rc);
}

static PyObject *synchronize_spin(PyObject *self, PyObject *arg) {
  (void)self;
  mgn_env *env = (mgn_env *)PyLong_AsVoidPtr(arg);
  if (PyErr_Occurred()) return NULL;
  if (env == NULL) {
    PyErr_SetString(PyExc_ValueError, "synchronize_spin: null handle");
    return NULL;
  }
  int rc;
  Py_BEGIN_ALLOW_THREADS rc = mgn_synchronize_spin(env);
  Py_END_ALLOW_THREADS return PyLong_FromLong(rc);
}

static PyMethodDef methods[] = {
    {"rollout", (PyCFunction)(void (*)(void))rollout, METH_FASTCALL,
     "mgn_rollout(env, actions, k, traj) -> int (MGN_OK = 0)"},
    {"synchronize", (PyCFunction)synchronize, METH_O, "mgn_synchronize(env) -> int (MGN_OK = 0)"},
    {"synchronize_spin", (PyCFunction)synchronize_spin, METH_O, "mgn_synchronize_spin(env) -> int (MGN_OK = 0)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_mgn_pycall", NULL, -1, methods};

PyMODINIT_FUNC PyInit__mgn_pycall(void) { return PyModule_Create(&module); }
