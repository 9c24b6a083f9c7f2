// gpx_lbfgsb_host.cpp — the reverse-communication L-BFGS-B loop of scipy's _minimize_lbfgsb
// (scipy 1.15, scipy/optimize/_lbfgsb_py.py), for a whole batch of fits in one host call.
//
// `gpflow.optimizers.Scipy().minimize` (GPR/model_trainer.py:18-19) runs scipy's L-BFGS-B: a
// Python loop around the compiled routine `setulb`, which asks for f and g at a point, takes
// them, and asks again until it reports convergence (or maxiter / maxfun stop it). The stepped
// drivers (optimizers.py) evaluate every fit's requested point in one batched device call, so
// per round each fit needs only its loop advanced to its next request. lbfgsb.LbfgsbStepper is
// that loop in Python (a generator per fit, ≈ 4 µs of interpreter work per evaluation); this
// module is the same loop in C++, over many fits per call, calling scipy's OWN `setulb` (passed
// in as the callable from scipy.optimize._lbfgsb) with the same arguments in the same sequence —
// so each fit's trajectory is scipy's bit for bit (tests/test_stream_driver.py checks against
// scipy.optimize.minimize and the Python stepper with atol = 0).
//
// Per slot the caller (lbfgsb.BatchStepper) creates scipy's work arrays once (x, bounds, nbd, g,
// wa, iwa, task, lsave, isave, dsave, ln_task: the dtypes and sizes _minimize_lbfgsb allocates);
// a fit started in a slot has them zeroed, as fresh arrays are. ScalarFunction's memoisation is
// kept: a requested point equal (element-wise ==) to the last evaluated one is answered from
// the stored f and g without a new evaluation, and nfev counts evaluations.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <cstring>
#include <vector>

namespace {

constexpr int kArgs = 17;  // setulb(m, x, l, u, nbd, f, g, factr, pgtol, wa, iwa, task, lsave, isave, dsave, maxls, ln_task)

enum : int { ST_IDLE = 0, ST_FIRST = 1, ST_WANT = 2, ST_DONE = 3 };

struct Slot {
  PyObject* args[kArgs] = {};
  Py_buffer buf[12] = {};  // x, l, u, nbd, g, wa, iwa, task, lsave, isave, dsave, ln_task
  bool have_buf = false;
  double* x = nullptr;
  double* g = nullptr;
  int32_t* task = nullptr;
  std::vector<double> sfx, sfg;  // ScalarFunction's x, g of the last evaluation
  double sff = 0.0;              // ... and its f
  double farg = 0.0;             // the f last passed to setulb
  long nfev = 0, nit = 0;
  int state = ST_IDLE;
};

struct BatchObject {
  PyObject_HEAD
  PyObject* setulb;
  int cap, n;
  long maxiter, maxfun;
  std::vector<Slot>* slots;
};

// a C-contiguous buffer of one element type ('i' int32, 'd' float64, 'B' / '?' bytes)
bool typed_buf(PyObject* o, Py_buffer* b, const char* fmts, Py_ssize_t item, bool writable, const char* what) {
  if (PyObject_GetBuffer(o, b, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT | (writable ? PyBUF_WRITABLE : 0)) != 0) return false;
  const char* f = b->format ? b->format : "B";
  if (*f == '<' || *f == '=' || *f == '@') ++f;
  if (b->itemsize != item || !std::strchr(fmts, *f) || f[1] != 0) {
    PyErr_Format(PyExc_TypeError, "%s: wrong element type (format %s, item size %zd)", what, b->format, b->itemsize);
    PyBuffer_Release(b);
    return false;
  }
  return true;
}

void release_slot(Slot& s) {
  for (auto& a : s.args) Py_CLEAR(a);
  if (s.have_buf)
    for (auto& b : s.buf) PyBuffer_Release(&b);
  s.have_buf = false;
}

void Batch_dealloc(BatchObject* self) {
  if (self->slots) {
    for (auto& s : *self->slots) release_slot(s);
    delete self->slots;
  }
  Py_XDECREF(self->setulb);
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

// Batch(setulb, cap, n, m, factr, pgtol, maxls, maxiter, maxfun, arrays): arrays[slot] = the 12
// work arrays of that slot, in the order of Slot::buf
int Batch_init(BatchObject* self, PyObject* args, PyObject*) {
  PyObject *setulb, *arrays;
  int cap, n, m, maxls;
  double factr, pgtol;
  long maxiter, maxfun;
  if (!PyArg_ParseTuple(args, "OiiiddillO", &setulb, &cap, &n, &m, &factr, &pgtol, &maxls, &maxiter, &maxfun,
                        &arrays))
    return -1;
  if (!PyCallable_Check(setulb) || cap <= 0 || n <= 0 || !PySequence_Check(arrays) ||
      PySequence_Size(arrays) != cap) {
    PyErr_SetString(PyExc_ValueError, "Batch: setulb must be callable and arrays hold one tuple per slot");
    return -1;
  }
  Py_INCREF(setulb);
  self->setulb = setulb;
  self->cap = cap;
  self->n = n;
  self->maxiter = maxiter;
  self->maxfun = maxfun;
  self->slots = new std::vector<Slot>(cap);
  static const int kArgOf[12] = {1, 2, 3, 4, 6, 9, 10, 11, 12, 13, 14, 16};  // buf index -> setulb argument
  static const Py_ssize_t kItem[12] = {8, 8, 8, 4, 8, 8, 4, 4, 4, 4, 8, 4};  // element bytes
  for (int i = 0; i < cap; ++i) {
    Slot& s = (*self->slots)[i];
    PyObject* t = PySequence_GetItem(arrays, i);
    if (!t) return -1;
    if (!PySequence_Check(t) || PySequence_Size(t) != 12) {
      Py_DECREF(t);
      PyErr_SetString(PyExc_ValueError, "Batch: each slot needs 12 work arrays");
      return -1;
    }
    int got = 0;
    for (int k = 0; k < 12; ++k) {
      PyObject* a = PySequence_GetItem(t, k);
      if (!a || !typed_buf(a, &s.buf[k], kItem[k] == 8 ? "d" : "i", kItem[k], true, "Batch: work array")) {
        Py_XDECREF(a);
        for (int j = 0; j < got; ++j) PyBuffer_Release(&s.buf[j]);
        Py_DECREF(t);
        return -1;
      }
      ++got;
      s.args[kArgOf[k]] = a;  // (the reference GetItem returned)
    }
    Py_DECREF(t);
    s.have_buf = true;
    if (s.buf[0].len != (Py_ssize_t)n * 8 || s.buf[4].len != (Py_ssize_t)n * 8 || s.buf[7].len != 8) {
      PyErr_SetString(PyExc_ValueError, "Batch: x / g must hold n float64, task two int32");
      return -1;
    }
    s.x = static_cast<double*>(s.buf[0].buf);
    s.g = static_cast<double*>(s.buf[4].buf);
    s.task = static_cast<int32_t*>(s.buf[7].buf);
    s.args[0] = PyLong_FromLong(m);
    s.args[5] = PyFloat_FromDouble(0.0);
    s.args[7] = PyFloat_FromDouble(factr);
    s.args[8] = PyFloat_FromDouble(pgtol);
    s.args[15] = PyLong_FromLong(maxls);
    if (!s.args[0] || !s.args[5] || !s.args[7] || !s.args[8] || !s.args[15]) return -1;
    s.sfx.assign(n, 0.0);
    s.sfg.assign(n, 0.0);
  }
  return 0;
}

Slot* slot_of(BatchObject* self, long i) {
  if (i < 0 || i >= self->cap) {
    PyErr_Format(PyExc_IndexError, "slot %ld out of range [0, %d)", i, self->cap);
    return nullptr;
  }
  return &(*self->slots)[i];
}

// f passed to setulb as a Python float (scipy passes its ScalarFunction's f)
int set_f(Slot& s, double f) {
  PyObject* o = PyFloat_FromDouble(f);
  if (!o) return -1;
  Py_SETREF(s.args[5], o);
  s.farg = f;
  return 0;
}

// Advance a slot whose (f, g) at sfx has just been stored: setulb until it wants f and g at a
// point other than sfx (state ST_WANT, sfx = that point) or stops (ST_DONE). -1 on a Python error.
int advance(BatchObject* self, Slot& s) {
  const int n = self->n;
  for (;;) {
    PyObject* r = PyObject_Vectorcall(self->setulb, s.args, kArgs, nullptr);
    if (!r) return -1;
    Py_DECREF(r);
    const int t0 = s.task[0];
    if (t0 == 3) {  // f and g wanted at x
      bool same = true;
      for (int i = 0; i < n; ++i) same = same && (s.x[i] == s.sfx[i]);
      if (!same) {
        std::memcpy(s.sfx.data(), s.x, sizeof(double) * n);
        s.state = ST_WANT;
        return 0;
      }
      if (set_f(s, s.sff) != 0) return -1;
      std::memcpy(s.g, s.sfg.data(), sizeof(double) * n);
    } else if (t0 == 1) {  // a new iteration
      s.nit += 1;
      if (s.nit >= self->maxiter) {
        s.task[0] = 5;
        s.task[1] = 504;
      } else if (s.nfev > self->maxfun) {
        s.task[0] = 5;
        s.task[1] = 502;
      }
    } else {
      s.state = ST_DONE;
      return 0;
    }
  }
}

// one evaluation's (f, g) into a slot that asked for it, then on to its next request
int tell_slot(BatchObject* self, Slot& s, double f, const double* g) {
  const int n = self->n;
  if (s.state != ST_FIRST && s.state != ST_WANT) {
    PyErr_SetString(PyExc_RuntimeError, "tell: the slot is not waiting for an evaluation");
    return -1;
  }
  s.nfev = s.state == ST_FIRST ? 1 : s.nfev + 1;
  s.sff = f;
  std::memcpy(s.sfg.data(), g, sizeof(double) * n);
  if (set_f(s, f) != 0) return -1;
  std::memcpy(s.g, g, sizeof(double) * n);
  return advance(self, s);
}

// start(slot, x0): a new fit in the slot (work arrays zeroed, x = x0); it asks for f, g at x0
PyObject* Batch_start(BatchObject* self, PyObject* args) {
  long i;
  PyObject* xo;
  Py_buffer xb;
  if (!PyArg_ParseTuple(args, "lO", &i, &xo) || !typed_buf(xo, &xb, "d", 8, false, "start: x0")) return nullptr;
  Slot* s = slot_of(self, i);
  if (!s || xb.len != (Py_ssize_t)self->n * 8) {
    if (s) PyErr_SetString(PyExc_ValueError, "start: x0 must hold n float64");
    PyBuffer_Release(&xb);
    return nullptr;
  }
  for (auto& b : s->buf) std::memset(b.buf, 0, b.len);
  std::memcpy(s->x, xb.buf, xb.len);
  std::memcpy(s->sfx.data(), xb.buf, xb.len);
  PyBuffer_Release(&xb);
  s->nfev = 0;
  s->nit = 0;
  s->state = ST_FIRST;
  if (set_f(*s, 0.0) != 0) return nullptr;  // (scipy's first pass: f = 0, g = 0)
  Py_RETURN_NONE;
}

// gather(rows int32[k], out float64[k, n]): the requested points
PyObject* Batch_gather(BatchObject* self, PyObject* args) {
  PyObject *ro, *oo;
  Py_buffer rb, ob;
  if (!PyArg_ParseTuple(args, "OO", &ro, &oo) || !typed_buf(ro, &rb, "i", 4, false, "gather: rows")) return nullptr;
  if (!typed_buf(oo, &ob, "d", 8, true, "gather: out")) {
    PyBuffer_Release(&rb);
    return nullptr;
  }
  const Py_ssize_t k = rb.len / 4;
  PyObject* ret = nullptr;
  if (ob.len != k * self->n * 8) {
    PyErr_SetString(PyExc_ValueError, "gather: rows int32[k], out float64[k, n]");
  } else {
    const int32_t* rows = static_cast<const int32_t*>(rb.buf);
    double* out = static_cast<double*>(ob.buf);
    bool ok = true;
    for (Py_ssize_t j = 0; j < k && ok; ++j) {
      Slot* s = slot_of(self, rows[j]);
      if (!s) ok = false;
      else std::memcpy(out + j * self->n, s->sfx.data(), sizeof(double) * self->n);
    }
    if (ok) ret = Py_NewRef(Py_None);
  }
  PyBuffer_Release(&rb);
  PyBuffer_Release(&ob);
  return ret;
}

// tell(rows int32[k], f float64[k], g float64[k, n], done uint8[k]): each row's evaluation, then
// its next request; done[j] = 1 when row j's fit has finished. On a Python error at row j the
// rows before it have been advanced (done[] says which finished), done[j] = 2, the rows after it
// are untouched and the error propagates.
PyObject* Batch_tell(BatchObject* self, PyObject* args) {
  PyObject *ro, *fo, *go, *dob;
  Py_buffer rb, fb, gb, db;
  if (!PyArg_ParseTuple(args, "OOOO", &ro, &fo, &go, &dob)) return nullptr;
  if (!typed_buf(ro, &rb, "i", 4, false, "tell: rows")) return nullptr;
  if (!typed_buf(fo, &fb, "d", 8, false, "tell: f")) {
    PyBuffer_Release(&rb);
    return nullptr;
  }
  if (!typed_buf(go, &gb, "d", 8, false, "tell: g")) {
    PyBuffer_Release(&rb);
    PyBuffer_Release(&fb);
    return nullptr;
  }
  if (!typed_buf(dob, &db, "B?", 1, true, "tell: done")) {
    PyBuffer_Release(&rb);
    PyBuffer_Release(&fb);
    PyBuffer_Release(&gb);
    return nullptr;
  }
  const Py_ssize_t k = rb.len / 4;
  PyObject* ret = nullptr;
  if (fb.len != k * 8 || gb.len != k * self->n * 8 || db.len != k) {
    PyErr_SetString(PyExc_ValueError, "tell: rows int32[k], f float64[k], g float64[k, n], done uint8[k]");
  } else {
    const int32_t* rows = static_cast<const int32_t*>(rb.buf);
    const double* f = static_cast<const double*>(fb.buf);
    const double* g = static_cast<const double*>(gb.buf);
    uint8_t* done = static_cast<uint8_t*>(db.buf);
    bool ok = true;
    for (Py_ssize_t j = 0; j < k && ok; ++j) {
      Slot* s = slot_of(self, rows[j]);
      ok = s && tell_slot(self, *s, f[j], g + j * self->n) == 0;
      done[j] = ok ? (s->state == ST_DONE) : 2;
    }
    if (ok) ret = Py_NewRef(Py_None);
  }
  PyBuffer_Release(&rb);
  PyBuffer_Release(&fb);
  PyBuffer_Release(&gb);
  PyBuffer_Release(&db);
  return ret;
}

// tell_one(slot, f, g): as tell for one fit; returns True when it has finished
PyObject* Batch_tell_one(BatchObject* self, PyObject* args) {
  long i;
  double f;
  PyObject* go;
  Py_buffer gb;
  if (!PyArg_ParseTuple(args, "ldO", &i, &f, &go) || !typed_buf(go, &gb, "d", 8, false, "tell_one: g")) return nullptr;
  Slot* s = slot_of(self, i);
  int rc = -1;
  if (s) {
    if (gb.len != (Py_ssize_t)self->n * 8) PyErr_SetString(PyExc_ValueError, "tell_one: g must hold n float64");
    else rc = tell_slot(self, *s, f, static_cast<const double*>(gb.buf));
  }
  PyBuffer_Release(&gb);
  if (rc != 0) return nullptr;
  return PyBool_FromLong(s->state == ST_DONE);
}

// state(slot) -> (state, nfev, nit, f last passed to setulb); the work arrays hold x, g, task, ...
PyObject* Batch_state(BatchObject* self, PyObject* args) {
  long i;
  if (!PyArg_ParseTuple(args, "l", &i)) return nullptr;
  Slot* s = slot_of(self, i);
  if (!s) return nullptr;
  return Py_BuildValue("(illd)", s->state, s->nfev, s->nit, s->farg);
}

// request(slot) -> the point the slot's fit wants evaluated (a new bytes object of n float64)
PyObject* Batch_request(BatchObject* self, PyObject* args) {
  long i;
  if (!PyArg_ParseTuple(args, "l", &i)) return nullptr;
  Slot* s = slot_of(self, i);
  if (!s) return nullptr;
  return PyBytes_FromStringAndSize(reinterpret_cast<const char*>(s->sfx.data()), sizeof(double) * self->n);
}

PyMethodDef Batch_methods[] = {
    {"start", (PyCFunction)Batch_start, METH_VARARGS, "start(slot, x0): a new fit in the slot"},
    {"gather", (PyCFunction)Batch_gather, METH_VARARGS, "gather(rows, out): the rows' requested points"},
    {"tell", (PyCFunction)Batch_tell, METH_VARARGS, "tell(rows, f, g, done): evaluations in, next requests out"},
    {"tell_one", (PyCFunction)Batch_tell_one, METH_VARARGS, "tell_one(slot, f, g) -> finished"},
    {"state", (PyCFunction)Batch_state, METH_VARARGS, "state(slot) -> (state, nfev, nit, f)"},
    {"request", (PyCFunction)Batch_request, METH_VARARGS, "request(slot) -> bytes of the requested point"},
    {nullptr, nullptr, 0, nullptr}};

PyTypeObject BatchType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyModuleDef module_def = {PyModuleDef_HEAD_INIT, "_gpx_lbfgsb",
                          "scipy's L-BFGS-B driver loop over a batch of fits (see gpx_lbfgsb_host.cpp)", -1,
                          nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__gpx_lbfgsb(void) {
  BatchType.tp_name = "_gpx_lbfgsb.Batch";
  BatchType.tp_basicsize = sizeof(BatchObject);
  BatchType.tp_flags = Py_TPFLAGS_DEFAULT;
  BatchType.tp_new = PyType_GenericNew;
  BatchType.tp_init = (initproc)Batch_init;
  BatchType.tp_dealloc = (destructor)Batch_dealloc;
  BatchType.tp_methods = Batch_methods;
  BatchType.tp_doc = "L-BFGS-B loop state of `cap` fits of dimension n (scipy's setulb per fit)";
  if (PyType_Ready(&BatchType) < 0) return nullptr;
  PyObject* mod = PyModule_Create(&module_def);
  if (!mod) return nullptr;
  Py_INCREF(&BatchType);
  if (PyModule_AddObject(mod, "Batch", reinterpret_cast<PyObject*>(&BatchType)) < 0) {
    Py_DECREF(&BatchType);
    Py_DECREF(mod);
    return nullptr;
  }
  return mod;
}
