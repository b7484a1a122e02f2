/* gym_lorenz._stepper: the per-env drop-in classes' hot call (envs/_single.py) as one
 * CPython C function instead of ctypes marshalling.  A Stepper holds the addresses of a
 * 1-env handle's host buffers (owned by the Python SingleEnvCore) and the address of
 * lz_resident_step / lz_step_host (include/lorenz_env.h); Stepper.step(action, noise)
 * writes the action (float32) and the optional injected noise (float64[3]) into those
 * buffers, makes the one C-ABI call and returns (obs copy, reward numpy scalar, done
 * byte as int) -- the values and types SingleEnvCore.step's ctypes path returns -- or the
 * lz_status int when the call fails (the caller raises through _native.check).
 *
 * Host marshalling only: the step itself runs in the HIP kernel behind the C-ABI.  Built
 * by gym-lorenz_amd/Makefile next to libgym_lorenz_amd.so; when it is missing the classes
 * use the ctypes call (same library, same results).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>
#include <stdint.h>
#include <string.h>

typedef int (*lz_step_fn)(void* h, const float* actions, const double* noise, void* obs_out,
                          void* rew_out, uint8_t* done_out);

typedef struct {
  PyObject_HEAD
  lz_step_fn fn;
  void* h;
  float* act;
  double* noise;
  void* obs;
  void* rew;
  uint8_t* done;
  int a_dim, o_dim, f64;
  PyArray_Descr* descr; /* float64 or float32: obs / reward dtype */
} Stepper;

static void Stepper_dealloc(Stepper* s) {
  Py_XDECREF(s->descr);
  Py_TYPE(s)->tp_free((PyObject*)s);
}

static int Stepper_init(Stepper* s, PyObject* args, PyObject* kw) {
  unsigned long long fn, h, act, noise, obs, rew, done;
  int a_dim, o_dim, f64;
  (void)kw;
  if (!PyArg_ParseTuple(args, "KKKKKKKiii", &fn, &h, &act, &noise, &obs, &rew, &done, &a_dim, &o_dim,
                        &f64))
    return -1;
  if (!fn || !h || !act || !noise || !obs || !rew || !done || a_dim < 0 || a_dim > 8 || o_dim < 1 ||
      o_dim > 64) {
    PyErr_SetString(PyExc_ValueError, "Stepper: bad addresses or dimensions");
    return -1;
  }
  s->fn = (lz_step_fn)(uintptr_t)fn;
  s->h = (void*)(uintptr_t)h;
  s->act = (float*)(uintptr_t)act;
  s->noise = (double*)(uintptr_t)noise;
  s->obs = (void*)(uintptr_t)obs;
  s->rew = (void*)(uintptr_t)rew;
  s->done = (uint8_t*)(uintptr_t)done;
  s->a_dim = a_dim;
  s->o_dim = o_dim;
  s->f64 = f64;
  Py_XDECREF(s->descr);
  s->descr = PyArray_DescrFromType(f64 ? NPY_FLOAT64 : NPY_FLOAT32);
  return s->descr ? 0 : -1;
}

/* n values of `obj` (an ndarray of any real dtype and shape with n elements, or a
 * sequence of n numbers) -> out[] as double; 0 on success, -1 with ValueError */
static int read_values(PyObject* obj, int n, double* out) {
  if (PyArray_Check(obj)) {
    PyArrayObject* a = (PyArrayObject*)obj;
    if (PyArray_SIZE(a) != n) goto bad;
    PyArrayObject* c = (PyArrayObject*)PyArray_FromAny(obj, PyArray_DescrFromType(NPY_FLOAT64), 0, 0,
                                                       NPY_ARRAY_CARRAY_RO | NPY_ARRAY_FORCECAST, NULL);
    if (!c) return -1;
    memcpy(out, PyArray_DATA(c), (size_t)n * sizeof(double));
    Py_DECREF(c);
    return 0;
  }
  {
    PyObject* seq = PySequence_Fast(obj, "expected a sequence");
    if (!seq) {
      PyErr_Clear();
      if (n == 1) { /* a bare number */
        out[0] = PyFloat_AsDouble(obj);
        return (out[0] == -1.0 && PyErr_Occurred()) ? -1 : 0;
      }
      goto bad;
    }
    if (PySequence_Fast_GET_SIZE(seq) != n) {
      Py_DECREF(seq);
      goto bad;
    }
    PyObject** items = PySequence_Fast_ITEMS(seq);
    for (int j = 0; j < n; ++j) {
      out[j] = PyFloat_AsDouble(items[j]);
      if (out[j] == -1.0 && PyErr_Occurred()) {
        Py_DECREF(seq);
        return -1;
      }
    }
    Py_DECREF(seq);
    return 0;
  }
bad:
  PyErr_Format(PyExc_ValueError, "expected %d values", n);
  return -1;
}

static PyObject* Stepper_step(Stepper* s, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs < 1 || nargs > 2) {
    PyErr_SetString(PyExc_TypeError, "step(action, noise=None)");
    return NULL;
  }
  double v[8];
  if (s->a_dim) {
    if (read_values(args[0], s->a_dim, v) != 0) return NULL;
    for (int j = 0; j < s->a_dim; ++j) s->act[j] = (float)v[j]; /* numpy's float32 cast */
  }
  const double* nz = NULL;
  if (nargs == 2 && args[1] != Py_None) {
    if (read_values(args[1], 3, s->noise) != 0) return NULL;
    nz = s->noise;
  }
  int st;
  Py_BEGIN_ALLOW_THREADS
  st = s->fn(s->h, s->act, nz, s->obs, s->rew, s->done);
  Py_END_ALLOW_THREADS
  if (st != 0) return PyLong_FromLong(st);
  npy_intp dim = s->o_dim;
  PyObject* obs = PyArray_SimpleNew(1, &dim, s->f64 ? NPY_FLOAT64 : NPY_FLOAT32);
  if (!obs) return NULL;
  memcpy(PyArray_DATA((PyArrayObject*)obs), s->obs, (size_t)s->o_dim * (s->f64 ? 8 : 4));
  PyObject* rew = PyArray_Scalar(s->rew, s->descr, NULL);
  if (!rew) {
    Py_DECREF(obs);
    return NULL;
  }
  PyObject* done = PyLong_FromLong((long)s->done[0]);
  if (!done) {
    Py_DECREF(obs);
    Py_DECREF(rew);
    return NULL;
  }
  PyObject* t = PyTuple_Pack(3, obs, rew, done);
  Py_DECREF(obs);
  Py_DECREF(rew);
  Py_DECREF(done);
  return t;
}

/* The handle is destroyed by its owner (SingleEnvCore.close -> lz_destroy): forget its
 * address, so a later step passes NULL and the library answers LZ_ERR_INVALID instead of
 * touching freed memory. */
static PyObject* Stepper_close(Stepper* s, PyObject* unused) {
  (void)unused;
  s->h = NULL;
  Py_RETURN_NONE;
}

static PyMethodDef Stepper_methods[] = {
    {"step", (PyCFunction)(void (*)(void))Stepper_step, METH_FASTCALL,
     "step(action, noise=None) -> (obs, reward, done) or an lz_status int"},
    {"close", (PyCFunction)Stepper_close, METH_NOARGS, "forget the handle (steps then fail cleanly)"},
    {NULL, NULL, 0, NULL}};

static PyTypeObject StepperType = {
    PyVarObject_HEAD_INIT(NULL, 0).tp_name = "gym_lorenz._stepper.Stepper",
    .tp_basicsize = sizeof(Stepper),
    .tp_flags = Py_TPFLAGS_DEFAULT,
    .tp_doc = "The per-env hot call (see lz_stepper.c)",
    .tp_new = PyType_GenericNew,
    .tp_init = (initproc)Stepper_init,
    .tp_dealloc = (destructor)Stepper_dealloc,
    .tp_methods = Stepper_methods,
};

static struct PyModuleDef stepper_module = {PyModuleDef_HEAD_INIT, "_stepper",
                                            "gym_lorenz per-env hot call", -1, NULL};

PyMODINIT_FUNC PyInit__stepper(void) {
  import_array();
  if (PyType_Ready(&StepperType) < 0) return NULL;
  PyObject* m = PyModule_Create(&stepper_module);
  if (!m) return NULL;
  Py_INCREF(&StepperType);
  if (PyModule_AddObject(m, "Stepper", (PyObject*)&StepperType) < 0) {
    Py_DECREF(&StepperType);
    Py_DECREF(m);
    return NULL;
  }
  return m;
}
