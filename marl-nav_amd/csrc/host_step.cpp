// _marlnav_host: the native host side of Env.step (marl-nav_amd/environment.py).
//
// The reference's Env.step (marlnav/environment.py:92-107) is a Python method;
// here its per-call host work - checking the actions tensor, picking the
// output tensors, filling the kernel's buffer table and enqueueing
// marlnav_step() (include/marlnav.h) on the current HIP stream - runs in C++,
// so that one call costs about as much as the kernel launch itself and the
// GPU, not the interpreter, sets the rate of a Python step loop.
//
// The engine owns a small pool of output sets. A set is the output of one
// step carved from ONE device allocation (packed observations, the fused
// normaliser's copy, reward, terminated, truncated) plus the Python objects
// handed out for it (the Observations tuple and its six views, the three
// tensors). A set is reused only when nothing outside the engine refers to
// it: every handed-out Python object is back at the reference count it had
// when the set was made, and no other tensor views its storage (the
// storage's use count is back at its baseline). A caller that keeps any
// output, or a view of one, therefore never sees it overwritten; otherwise
// the memory is recycled and a step allocates nothing.
//
// Everything else (parameter sync, state-buffer replacement, the reference-
// RNG and mock-initializer modes, action coercion) stays in Python and talks
// to the engine through configure()/launch().
#include <Python.h>
#include <structmember.h>

#include <torch/csrc/autograd/python_variable.h>

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

#include "../../include/marlnav.h"

namespace {

constexpr int kMaxObjs = 16;
constexpr int kPoolMax = 4;

using StepFn = int (*)(const MarlnavDims *, const MarlnavParams *, const MarlnavStepBuffers *,
                       uint64_t, void *);
using ErrFn = const char *(*)(void);

struct OutSet {
    PyObject *obs = nullptr;          // _PackedObservations
    PyObject *reward = nullptr;       // (P,) f32
    PyObject *terminated = nullptr;   // (P,) bool
    PyObject *truncated = nullptr;    // (P,) bool
    PyObject *objs[kMaxObjs] = {};    // every handed-out object (strong refs)
    Py_ssize_t base[kMaxObjs] = {};   // their reference counts when only the set held them
    int nobj = 0;
    c10::Storage storage;             // the set's one allocation
    size_t base_use = 0;
    void *obs_ptr = nullptr, *reward_ptr = nullptr, *term_ptr = nullptr, *trunc_ptr = nullptr,
         *norm_ptr = nullptr;
    bool pooled = false;

    bool is_free() const
    {
        if (storage.use_count() != base_use) return false;
        for (int i = 0; i < nobj; ++i)
            if (Py_REFCNT(objs[i]) != base[i]) return false;
        return true;
    }
    void release()
    {
        for (int i = 0; i < nobj; ++i) Py_CLEAR(objs[i]);
        nobj = 0;
        Py_CLEAR(obs);
        Py_CLEAR(reward);
        Py_CLEAR(terminated);
        Py_CLEAR(truncated);
        storage = c10::Storage();
    }
};

// tensors of the Env that a step writes (track_state): states, obstacles,
// target, step_num, terminates, and the second states buffer
constexpr int kHeld = 6;
constexpr int kStates = 0, kStatesAlt = 5;
// Python references a tracked tensor has when nothing outside the Env holds
// it: the Env attribute and this engine, except the two state buffers, which
// only the engine holds (Env.states asks the engine for the current one)
constexpr Py_ssize_t kOwnRefs[kHeld] = {1, 2, 2, 2, 2, 1};

struct Engine {
    PyObject_HEAD
    MarlnavDims dims;
    MarlnavParams params;
    MarlnavStepBuffers base;      // state buffers, formation, counters, normaliser
    StepFn step_fn;
    ErrFn err_fn;
    PyObject *stream_fn;          // torch._C._cuda_getCurrentRawStream
    PyObject *dev_index;          // int
    PyObject *factory;            // () -> (obs, reward, terminated, truncated, packed, normalized|None)
    PyObject *slow_step;          // Env._step_py(actions): coercion / params / reference modes
    int device;
    int64_t act_shape[3];
    int fast_ok;                  // native re-init, default sampler, params in sync
    int write_norm;               // sets carry a normaliser output
    int allow_capture;            // launches under stream capture accepted (timing)
    unsigned long long step_idx;  // native RNG step counter (environment.py:92 call count + 1)
    unsigned long long steps_done;
    std::vector<OutSet *> *pool;
    int next;
    OutSet *last;                 // the set the previous step returned
    // the Env's states / obstacles / target / step_num / terminates tensors
    // (strong refs, track_state): a step may not write them in place while
    // anything else refers to them
    PyObject *held[kHeld];
    c10::Storage held_st[kHeld];
};

// The reference's re-init rebinds `states`, `obstacles`, `target` and
// `_step_num` to new tensors (environment.py:79-83) and `_terminates` at
// :219, so a caller holding the old tensor keeps its pre-step values (for
// `states`: the moved ones, :113-123 move in place; for `_step_num`: +1, the
// in-place increment of :96). Here the step kernel writes them in place, so the step goes
// through Env._step_py, which gives the Env fresh copies first, whenever a
// tensor is referenced beyond the Env's attribute and this engine (2 Python
// references) or its storage is viewed by another tensor (use count beyond
// the tensor's own and this engine's copy).
bool state_shared(const Engine *e, int i)
{
    return e->held[i] &&
           (Py_REFCNT(e->held[i]) > kOwnRefs[i] || e->held_st[i].use_count() > 2);
}

bool any_state_shared(const Engine *e)
{
    for (int i = 0; i < kHeld; ++i)
        if (state_shared(e, i)) return true;
    return false;
}

void release_state(Engine *e)
{
    for (int i = 0; i < kHeld; ++i) {
        Py_CLEAR(e->held[i]);
        e->held_st[i] = c10::Storage();
    }
}

PyObject *raise_step_error(Engine *e, int rc)
{
    const char *msg = e->err_fn ? e->err_fn() : nullptr;
    PyErr_Format(PyExc_RuntimeError, "marlnav error %d: %s", rc, msg ? msg : "?");
    return nullptr;
}

// Build a set through the Python factory; its objects' reference counts
// right after the factory's frame is gone are the 'held by the pool only'
// baseline.
OutSet *make_set(Engine *e)
{
    PyObject *t = PyObject_CallNoArgs(e->factory);
    if (!t) return nullptr;
    if (!PyTuple_Check(t) || PyTuple_GET_SIZE(t) != 6) {
        Py_DECREF(t);
        PyErr_SetString(PyExc_TypeError, "output-set factory must return a 6-tuple");
        return nullptr;
    }
    OutSet *s = new OutSet();
    PyObject *obs = PyTuple_GET_ITEM(t, 0), *packed = PyTuple_GET_ITEM(t, 4),
             *norm = PyTuple_GET_ITEM(t, 5);
    s->obs = obs;
    s->reward = PyTuple_GET_ITEM(t, 1);
    s->terminated = PyTuple_GET_ITEM(t, 2);
    s->truncated = PyTuple_GET_ITEM(t, 3);
    Py_INCREF(s->obs);
    Py_INCREF(s->reward);
    Py_INCREF(s->terminated);
    Py_INCREF(s->truncated);
    auto track = [s](PyObject *o) {
        Py_INCREF(o);
        s->objs[s->nobj++] = o;
    };
    track(obs);
    track(s->reward);
    track(s->terminated);
    track(s->truncated);
    track(packed);
    if (norm != Py_None) track(norm);
    const Py_ssize_t nf = PyTuple_Check(obs) ? PyTuple_GET_SIZE(obs) : 0;
    for (Py_ssize_t i = 0; i < nf && s->nobj < kMaxObjs; ++i) track(PyTuple_GET_ITEM(obs, i));
    for (int i = 0; i < s->nobj; ++i)
        if (!THPVariable_Check(s->objs[i]) && s->objs[i] != obs) {
            Py_DECREF(t);
            s->release();
            delete s;
            PyErr_SetString(PyExc_TypeError, "output-set factory returned a non-tensor");
            return nullptr;
        }
    const at::Tensor &pk = THPVariable_Unpack(packed);
    s->obs_ptr = pk.data_ptr();
    s->reward_ptr = THPVariable_Unpack(s->reward).data_ptr();
    s->term_ptr = THPVariable_Unpack(s->terminated).data_ptr();
    s->trunc_ptr = THPVariable_Unpack(s->truncated).data_ptr();
    s->norm_ptr = norm != Py_None ? THPVariable_Unpack(norm).data_ptr() : nullptr;
    s->storage = pk.storage();
    Py_DECREF(t);
    s->base_use = s->storage.use_count();
    for (int i = 0; i < s->nobj; ++i) s->base[i] = Py_REFCNT(s->objs[i]);
    return s;
}

void clear_pool(Engine *e)
{
    if (!e->pool) return;
    if (e->last && !e->last->pooled) {
        e->last->release();
        delete e->last;
    }
    e->last = nullptr;
    for (OutSet *s : *e->pool) {
        s->release();
        delete s;
    }
    e->pool->clear();
    e->next = 0;
}

// The set this step writes: a pooled one nothing references any more, else
// a new allocation (pooled while the pool is small; never while capturing).
OutSet *take_set(Engine *e, bool capturing)
{
    std::vector<OutSet *> &pool = *e->pool;
    const int n = (int)pool.size();
    if (n && !capturing) {
        int i = e->next;
        for (int k = 0; k < (n > 1 ? 2 : 1); ++k) {
            OutSet *s = pool[i];
            i = i + 1 < n ? i + 1 : 0;
            if (s != e->last && s->is_free()) {
                e->next = i;
                return s;
            }
        }
    }
    OutSet *s = make_set(e);
    if (!s) return nullptr;
    if (!capturing && n < kPoolMax) {
        s->pooled = true;
        pool.push_back(s);
    }
    return s;
}

void forget_last(Engine *e)
{
    if (e->last && !e->last->pooled) {
        e->last->release();
        delete e->last;
    }
    e->last = nullptr;
}

bool current_stream(Engine *e, void **stream)
{
    PyObject *r = PyObject_CallOneArg(e->stream_fn, e->dev_index);
    if (!r) return false;
    *stream = PyLong_AsVoidPtr(r);
    Py_DECREF(r);
    return !PyErr_Occurred();
}

// One marlnav_step launch with the given actions (and, for the reference-
// RNG / mock modes, fresh candidates and extra flags); returns the step's
// (obs, reward, terminated, truncated).
PyObject *do_launch(Engine *e, const void *actions, const MarlnavStepBuffers *fresh,
                    uint32_t extra_flags)
{
    void *stream = nullptr;
    if (!current_stream(e, &stream)) return nullptr;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)stream, &cap) != hipSuccess) {
        (void)hipGetLastError();
        cap = hipStreamCaptureStatusNone;
    }
    const bool capturing = cap == hipStreamCaptureStatusActive;
    if (capturing && !e->allow_capture) {
        // a captured step bakes this call's RNG step index (native re-init)
        // or fresh candidates (reference RNG) into the graph: every replay
        // would re-initialise finished envs with the same draws
        PyErr_SetString(PyExc_RuntimeError,
                        "Env.step under stream capture replays this step's re-init draws on "
                        "every graph replay; set env.allow_graph_capture = True to accept "
                        "that (timing runs)");
        return nullptr;
    }
    if (capturing && e->base.states_out && e->held[kStatesAlt]) {
        // double-buffered states swap roles on the host once per call: a
        // capture records the swap once, so every replay would read the same
        // buffer and write the other, and the states would never advance
        PyErr_SetString(PyExc_RuntimeError,
                        "Env.step under stream capture is not supported with double-buffered "
                        "states (states_double_buffer=True): the buffer swap happens on the host");
        return nullptr;
    }
    OutSet *s = take_set(e, capturing);
    if (!s) return nullptr;
    MarlnavStepBuffers b = e->base;
    b.actions = (const float *)actions;
    b.obs = (float *)s->obs_ptr;
    b.reward = (float *)s->reward_ptr;
    b.terminated = (uint8_t *)s->term_ptr;
    b.truncated = (uint8_t *)s->trunc_ptr;
    uint32_t flags = e->params.flags & ~(uint32_t)(MARLNAV_FRESH_STATES_FROM_MOVED |
                                                   MARLNAV_WRITE_OBS_NORM);
    if (s->norm_ptr) {
        b.obs_norm = (float *)s->norm_ptr;
        flags |= MARLNAV_WRITE_OBS_NORM;
    } else {
        b.obs_norm = nullptr;
    }
    if (fresh) {
        b.fresh_states = fresh->fresh_states;
        b.fresh_obstacles = fresh->fresh_obstacles;
        b.fresh_target = fresh->fresh_target;
    } else {
        b.fresh_states = b.fresh_obstacles = b.fresh_target = nullptr;
    }
    MarlnavParams p = e->params;
    p.flags = flags | extra_flags;
    const int rc = e->step_fn(&e->dims, &p, &b, e->step_idx, stream);
    if (rc) {
        if (!s->pooled) {
            s->release();
            delete s;
        }
        return raise_step_error(e, rc);
    }
    if (b.states_out && e->held[kStatesAlt]) {
        // the step wrote the new states into the second buffer: it is the
        // current one from here on
        std::swap(e->held[kStates], e->held[kStatesAlt]);
        std::swap(e->held_st[kStates], e->held_st[kStatesAlt]);
        std::swap(e->base.states, e->base.states_out);
    }
    e->step_idx++;
    e->steps_done++;
    if (e->last != s) forget_last(e);
    e->last = s;
    return PyTuple_Pack(4, s->obs, s->reward, s->terminated, s->truncated);
}

// ------------------------------------------------------------ Python type

int Engine_init(Engine *e, PyObject *args, PyObject *)
{
    unsigned long long step_addr = 0, err_addr = 0;
    PyObject *stream_fn, *factory, *slow;
    int device;
    if (!PyArg_ParseTuple(args, "KKOiOO", &step_addr, &err_addr, &stream_fn, &device, &factory,
                          &slow))
        return -1;
    if (!step_addr || !PyCallable_Check(stream_fn) || !PyCallable_Check(factory) ||
        !PyCallable_Check(slow)) {
        PyErr_SetString(PyExc_TypeError, "Engine(step_fn, err_fn, stream_fn, device, factory, slow)");
        return -1;
    }
    e->step_fn = reinterpret_cast<StepFn>(step_addr);
    e->err_fn = reinterpret_cast<ErrFn>(err_addr);
    Py_INCREF(stream_fn);
    e->stream_fn = stream_fn;
    e->dev_index = PyLong_FromLong(device);
    e->device = device;
    Py_INCREF(factory);
    e->factory = factory;
    Py_INCREF(slow);
    e->slow_step = slow;
    e->pool = new std::vector<OutSet *>();
    memset(&e->dims, 0, sizeof(e->dims));
    memset(&e->params, 0, sizeof(e->params));
    memset(&e->base, 0, sizeof(e->base));
    e->fast_ok = 0;
    e->write_norm = 0;
    e->allow_capture = 0;
    e->step_idx = 1;
    e->steps_done = 0;
    e->next = 0;
    e->last = nullptr;
    for (int i = 0; i < kHeld; ++i) {
        e->held[i] = nullptr;
        new (&e->held_st[i]) c10::Storage();
    }
    return e->dev_index ? 0 : -1;
}

void Engine_dealloc(Engine *e)
{
    clear_pool(e);
    delete e->pool;
    release_state(e);
    for (int i = 0; i < kHeld; ++i) e->held_st[i].~Storage();
    Py_CLEAR(e->stream_fn);
    Py_CLEAR(e->dev_index);
    Py_CLEAR(e->factory);
    Py_CLEAR(e->slow_step);
    Py_TYPE(e)->tp_free((PyObject *)e);
}

bool read_struct(PyObject *o, void *dst, size_t n, const char *what)
{
    Py_buffer v;
    if (PyObject_GetBuffer(o, &v, PyBUF_SIMPLE) < 0) return false;
    const bool ok = (size_t)v.len == n;
    if (ok) memcpy(dst, v.buf, n);
    PyBuffer_Release(&v);
    if (!ok) PyErr_Format(PyExc_ValueError, "%s: expected %zu bytes", what, n);
    return ok;
}

// configure(dims, params, base_buffers, fast_ok): the structs as bytes-like
// objects (ctypes structures of marl-nav_amd/abi.py).
PyObject *Engine_configure(Engine *e, PyObject *args)
{
    PyObject *d, *p, *b;
    int fast_ok;
    if (!PyArg_ParseTuple(args, "OOOp", &d, &p, &b, &fast_ok)) return nullptr;
    MarlnavDims nd;
    if (!read_struct(d, &nd, sizeof nd, "dims") || !read_struct(p, &e->params, sizeof e->params, "params") ||
        !read_struct(b, &e->base, sizeof e->base, "buffers"))
        return nullptr;
    e->dims = nd;
    const int D = 2 + 2 * nd.num_obstacles + 2 * (nd.num_agents - 1);
    (void)D;
    e->act_shape[0] = nd.num_parallel;
    e->act_shape[1] = nd.num_agents;
    e->act_shape[2] = 2;
    e->fast_ok = fast_ok;
    Py_RETURN_NONE;
}

// The fast path: native re-init, default sampler, params in sync, actions
// already an f32 contiguous 16-byte-aligned (P, A, 2) tensor on the env's
// device. Anything
// else goes through Env._step_py (Python), which coerces and then comes back
// through launch().
PyObject *Engine_call(Engine *e, PyObject *args, PyObject *kw)
{
    PyObject *a;
    if (kw || !PyTuple_Check(args) || PyTuple_GET_SIZE(args) != 1) {
        PyErr_SetString(PyExc_TypeError, "step(actions)");
        return nullptr;
    }
    a = PyTuple_GET_ITEM(args, 0);
    if (e->fast_ok && !any_state_shared(e) && THPVariable_Check(a)) {
        const at::Tensor &t = THPVariable_Unpack(a);
        if (t.scalar_type() == at::kFloat && t.dim() == 3 && t.is_cuda() &&
            t.get_device() == e->device && t.size(0) == e->act_shape[0] &&
            t.size(1) == e->act_shape[1] && t.size(2) == 2 && t.is_contiguous() &&
            !t.requires_grad() && (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15u) == 0)
            return do_launch(e, t.data_ptr(), nullptr, 0);
    }
    return PyObject_CallOneArg(e->slow_step, a);
}

// launch(actions, fresh_ptrs_or_None, extra_flags): used by Env._step_py
// after coercion; fresh_ptrs = (states, obstacles, target) device pointers.
PyObject *Engine_launch(Engine *e, PyObject *args)
{
    unsigned long long act;
    PyObject *fresh;
    unsigned int extra;
    if (!PyArg_ParseTuple(args, "KOI", &act, &fresh, &extra)) return nullptr;
    MarlnavStepBuffers f;
    memset(&f, 0, sizeof f);
    const MarlnavStepBuffers *fp = nullptr;
    if (fresh != Py_None) {
        unsigned long long s, o, t;
        if (!PyArg_ParseTuple(fresh, "KKK", &s, &o, &t)) return nullptr;
        f.fresh_states = (const float *)s;
        f.fresh_obstacles = (const float *)o;
        f.fresh_target = (const float *)t;
        fp = &f;
    }
    return do_launch(e, (const void *)act, fp, extra);
}

// track_state(states, obstacles, target, step_num, terminates, states_alt):
// the Env's current tensors; states_alt (or None) is the buffer the next step
// writes the new states into (MarlnavStepBuffers.states_out), after which
// the two state buffers swap roles (double-buffered states: the step never
// writes the lines it read)
PyObject *Engine_track_state(Engine *e, PyObject *args)
{
    PyObject *o[kHeld];
    if (!PyArg_ParseTuple(args, "OOOOOO", &o[0], &o[1], &o[2], &o[3], &o[4], &o[5]))
        return nullptr;
    for (int i = 0; i < kHeld; ++i)
        if (!THPVariable_Check(o[i]) && !(i == kStatesAlt && o[i] == Py_None)) {
            PyErr_SetString(PyExc_TypeError,
                            "track_state(states, obstacles, target, step_num, terminates, "
                            "states_alt|None): tensors");
            return nullptr;
        }
    release_state(e);
    for (int i = 0; i < kHeld; ++i) {
        if (o[i] == Py_None) continue;
        Py_INCREF(o[i]);
        e->held[i] = o[i];
        e->held_st[i] = THPVariable_Unpack(o[i]).storage();
    }
    e->base.states = e->held[kStates] ? (float *)THPVariable_Unpack(e->held[kStates]).data_ptr()
                                      : e->base.states;
    e->base.states_out = e->held[kStatesAlt]
                             ? (float *)THPVariable_Unpack(e->held[kStatesAlt]).data_ptr()
                             : nullptr;
    Py_RETURN_NONE;
}

// the current states tensor (new reference), or None
PyObject *Engine_states(Engine *e, PyObject *)
{
    PyObject *t = e->held[kStates] ? e->held[kStates] : Py_None;
    Py_INCREF(t);
    return t;
}

// the second states buffer (new reference), or None
PyObject *Engine_states_alt(Engine *e, PyObject *)
{
    PyObject *t = e->held[kStatesAlt] ? e->held[kStatesAlt] : Py_None;
    Py_INCREF(t);
    return t;
}

// one flag per tracked tensor: (states, obstacles, target, step_num, terminates)
PyObject *Engine_shared_state(Engine *e, PyObject *)
{
    PyObject *t = PyTuple_New(kHeld);
    for (int i = 0; i < kHeld; ++i) {
        PyObject *b = state_shared(e, i) ? Py_True : Py_False;
        Py_INCREF(b);
        PyTuple_SET_ITEM(t, i, b);
    }
    return t;
}

PyObject *Engine_reset_pool(Engine *e, PyObject *)
{
    clear_pool(e);
    Py_RETURN_NONE;
}

// (terminated, truncated) of the last step, or None
PyObject *Engine_last_finished(Engine *e, PyObject *)
{
    if (!e->last) Py_RETURN_NONE;
    return PyTuple_Pack(2, e->last->terminated, e->last->truncated);
}

PyObject *Engine_pool_info(Engine *e, PyObject *)
{
    PyObject *l = PyList_New(0);
    for (OutSet *s : *e->pool) {
        PyObject *x = Py_BuildValue("(KO)", (unsigned long long)(uintptr_t)s->obs_ptr,
                                    s->is_free() ? Py_True : Py_False);
        PyList_Append(l, x);
        Py_DECREF(x);
    }
    return l;
}

PyMethodDef Engine_methods[] = {
    {"configure", (PyCFunction)Engine_configure, METH_VARARGS,
     "configure(dims, params, buffers, fast_ok)"},
    {"launch", (PyCFunction)Engine_launch, METH_VARARGS,
     "launch(actions_ptr, fresh_ptrs|None, extra_flags) -> (obs, reward, terminated, truncated)"},
    {"reset_pool", (PyCFunction)Engine_reset_pool, METH_NOARGS, "drop every pooled output set"},
    {"track_state", (PyCFunction)Engine_track_state, METH_VARARGS,
     "track_state(states, obstacles, target, step_num, terminates, states_alt|None): the tensors a "
     "step must not write while shared"},
    {"shared_state", (PyCFunction)Engine_shared_state, METH_NOARGS,
     "(states, obstacles, target, step_num, terminates, states_alt) shared flags"},
    {"states", (PyCFunction)Engine_states, METH_NOARGS, "the current states tensor"},
    {"states_alt", (PyCFunction)Engine_states_alt, METH_NOARGS,
     "the buffer the next step writes the states into, or None"},
    {"last_finished", (PyCFunction)Engine_last_finished, METH_NOARGS,
     "(terminated, truncated) of the last step or None"},
    {"pool_info", (PyCFunction)Engine_pool_info, METH_NOARGS, "[(obs_ptr, free)] per pooled set"},
    {nullptr, nullptr, 0, nullptr}};

PyMemberDef Engine_members[] = {
    {"step_idx", T_ULONGLONG, offsetof(Engine, step_idx), 0, "native RNG step counter"},
    {"steps_done", T_ULONGLONG, offsetof(Engine, steps_done), READONLY, "launched steps"},
    {"fast_ok", T_INT, offsetof(Engine, fast_ok), 0, "fast path enabled"},
    {"allow_capture", T_INT, offsetof(Engine, allow_capture), 0,
     "accept launches under stream capture"},
    {nullptr, 0, 0, 0, nullptr}};

PyTypeObject EngineType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyModuleDef module_def = {PyModuleDef_HEAD_INIT, "_marlnav_host",
                          "Native host side of marlnav_amd.Env.step", -1, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__marlnav_host(void)
{
    EngineType.tp_name = "_marlnav_host.Engine";
    EngineType.tp_basicsize = sizeof(Engine);
    EngineType.tp_flags = Py_TPFLAGS_DEFAULT;
    EngineType.tp_new = PyType_GenericNew;
    EngineType.tp_init = (initproc)Engine_init;
    EngineType.tp_dealloc = (destructor)Engine_dealloc;
    EngineType.tp_call = (ternaryfunc)Engine_call;
    EngineType.tp_methods = Engine_methods;
    EngineType.tp_members = Engine_members;
    EngineType.tp_doc = "Env.step host engine: step(actions) -> (obs, reward, terminated, truncated)";
    if (PyType_Ready(&EngineType) < 0) return nullptr;
    PyObject *m = PyModule_Create(&module_def);
    if (!m) return nullptr;
    Py_INCREF(&EngineType);
    if (PyModule_AddObject(m, "Engine", (PyObject *)&EngineType) < 0) {
        Py_DECREF(&EngineType);
        Py_DECREF(m);
        return nullptr;
    }
    PyModule_AddIntConstant(m, "POOL_MAX", kPoolMax);
    return m;
}
