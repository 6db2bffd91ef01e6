"""No-code reader of the reference's quantized SuperPoint TorchScript archives
(python/superpoint_quantized_nonorm.pt, python/superpoint_quantized.pt; built by
python/superpoint_inference.py:29-83's SuperPointNet, loaded there by torch.load at :110-114).

The archive is a zip: `<name>/data.pkl` (the module tree as a pickle), `<name>/data/<key>` (raw
tensor storages) and `<name>/code/` (TorchScript source).  This module NEVER unpickles and never
runs TorchScript: `data.pkl` is walked opcode by opcode (pickletools.genops) by a small stack
machine in which GLOBAL only names a symbol, REDUCE / NEWOBJ / BUILD only record what they would
call, and BINPERSID only records the storage key -- nothing named in the file is imported or
called.  The recorded tree is then read as the quantized Conv2d state tuples
(torch/ao/nn/quantized/modules/conv.py __setstate__: in/out channels, kernel, stride, padding,
dilation, transposed, output padding, groups, padding mode, weight, bias, output scale, output
zero point, training), the weights as `_rebuild_qtensor(storage, offset, size, stride,
(per_tensor_affine, scale, zero_point), ...)` over int8 storages, the biases as
`_rebuild_tensor_v2` over float32 storages, and the input Quantize module's scale / zero-point
buffers.  Anything outside that shape raises."""
import io
import pickletools
import zipfile

import numpy as np

LAYERS = ("conv1a", "conv1b", "conv2a", "conv2b", "conv3a", "conv3b", "conv4a", "conv4b",
          "convPa", "convPb", "convDa", "convDb")


class Global:
    def __init__(self, module, name):
        self.module, self.name = module, name

    def __repr__(self):
        return "Global(%s.%s)" % (self.module, self.name)


class Call:  # func(*args), recorded, never performed
    def __init__(self, func, args):
        self.func, self.args = func, args


class Obj:  # cls.__new__(cls, *args) then __setstate__(state), recorded
    def __init__(self, cls, args):
        self.cls, self.args, self.state = cls, args, None


class PersId:
    def __init__(self, pid):
        self.pid = pid


_MARK = object()


def walk_pickle(data):
    """The pickle's object graph with every callable left as a record (see module docstring)."""
    stack, memo = [], {}

    def pop_mark():
        k = len(stack) - 1
        while stack[k] is not _MARK:
            k -= 1
        items = stack[k + 1:]
        del stack[k:]
        return items

    for op, arg, _pos in pickletools.genops(io.BytesIO(data)):
        n = op.name
        if n == "PROTO":
            continue
        if n == "GLOBAL":
            mod, name = arg.split(" ", 1)
            stack.append(Global(mod, name))
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n == "MARK":
            stack.append(_MARK)
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            items = tuple(stack[-k:])
            del stack[-k:]
            stack.append(items)
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif n == "APPENDS":
            items = pop_mark()
            stack[-1].extend(items)
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif n == "SETITEMS":
            items = pop_mark()
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif n in ("BININT", "BININT1", "BININT2", "LONG1", "INT"):
            stack.append(int(arg))
        elif n == "BINFLOAT":
            stack.append(float(arg))
        elif n in ("BINUNICODE", "SHORT_BINUNICODE", "UNICODE"):
            stack.append(str(arg))
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWOBJ":
            args = stack.pop()
            cls = stack.pop()
            stack.append(Obj(cls, args))
        elif n == "REDUCE":
            args = stack.pop()
            func = stack.pop()
            stack.append(Call(func, args))
        elif n == "BUILD":
            state = stack.pop()
            if not isinstance(stack[-1], Obj):
                raise ValueError("BUILD on a non-object record")
            stack[-1].state = state
        elif n == "BINPERSID":
            stack.append(PersId(stack.pop()))
        elif n == "STOP":
            if len(stack) != 1:
                raise ValueError("malformed pickle stack")
            return stack[0]
        else:
            raise ValueError("opcode %s outside the reader's subset" % n)
    raise ValueError("no STOP opcode")


_STORAGE_DTYPES = {"QInt8Storage": np.int8, "FloatStorage": np.float32, "LongStorage": np.int64,
                   "ByteStorage": np.uint8, "IntStorage": np.int32, "DoubleStorage": np.float64}


def _is_global(g, module, name):
    return isinstance(g, Global) and g.module == module and g.name == name


class _Archive:
    def __init__(self, path):
        self.z = zipfile.ZipFile(path)
        pkls = [n for n in self.z.namelist() if n.endswith("/data.pkl") and n.count("/") == 1]
        if len(pkls) != 1:
            raise ValueError("%s: expected one <name>/data.pkl" % path)
        self.prefix = pkls[0][:-len("data.pkl")]

    def storage(self, pid):
        if not (isinstance(pid, tuple) and len(pid) == 5 and pid[0] == "storage" and isinstance(pid[1], Global)
                and pid[1].module == "torch" and pid[1].name in _STORAGE_DTYPES):
            raise ValueError("unexpected persistent id %r" % (pid,))
        dt = np.dtype(_STORAGE_DTYPES[pid[1].name]).newbyteorder("<")
        raw = self.z.read(self.prefix + "data/" + pid[2])
        a = np.frombuffer(raw, dtype=dt)
        if a.size != pid[4]:
            raise ValueError("storage %s: %d elements, %d recorded" % (pid[2], a.size, pid[4]))
        return a

    def tensor(self, rec):
        """(array, quantizer) of a `_rebuild_qtensor` / `_rebuild_tensor_v2` record"""
        if not isinstance(rec, Call) or not isinstance(rec.func, Global) or rec.func.module != "torch._utils":
            raise ValueError("unexpected tensor record")
        a = rec.args
        st = self.storage(a[0].pid)
        off, size, stride = a[1], tuple(a[2]), tuple(a[3])
        end = off + sum((s - 1) * t for s, t in zip(size, stride)) + 1 if size else off + 1
        if min(size, default=1) > 0 and (off < 0 or end > st.size):
            raise ValueError("tensor view outside its storage")
        view = np.lib.stride_tricks.as_strided(st[off:], shape=size, strides=[t * st.itemsize for t in stride])
        arr = np.ascontiguousarray(view)
        if rec.func.name == "_rebuild_qtensor":
            q = a[4]
            if not (_is_global(q[0], "torch", "per_tensor_affine") and len(q) == 3):
                raise ValueError("only per-tensor affine quantisation is read (found %r)" % (q[0],))
            return arr, (float(q[1]), int(q[2]))
        if rec.func.name == "_rebuild_tensor_v2":
            return arr, None
        raise ValueError("unexpected rebuild function %s" % rec.func.name)


def load_superpoint(path):
    """Layer table of a quantized SuperPoint archive:
    {'input': {'scale', 'zero_point', 'dtype'},
     'conv1a' ... 'convDb': {'w' int8 [Cout][Cin][kh][kw], 'w_scale', 'w_zp', 'bias' float32 [Cout],
                             'out_scale', 'out_zp', 'stride', 'padding', 'kernel'}}"""
    ar = _Archive(path)
    root = walk_pickle(ar.z.read(ar.prefix + "data.pkl"))
    if not (isinstance(root, Obj) and root.cls.name == "SuperPointNet" and isinstance(root.state, dict)):
        raise ValueError("not a SuperPointNet archive")
    out = {}
    for name in LAYERS:
        m = root.state[name]
        if not (isinstance(m, Obj) and m.cls.name == "Conv2d" and "quantized" in m.cls.module):
            raise ValueError("%s: not a quantized Conv2d" % name)
        s = m.state
        cin, cout, ks, stride, pad, dil, transposed, _opad, groups, mode = s[:10]
        if transposed or groups != 1 or tuple(dil) != (1, 1) or mode != "zeros":
            raise ValueError("%s: unsupported conv configuration" % name)
        w, (ws, wz) = ar.tensor(s[10])
        b, _ = ar.tensor(s[11]) if s[11] is not None else (np.zeros(cout, np.float32), None)
        if w.shape != (cout, cin) + tuple(ks) or w.dtype != np.int8 or b.shape != (cout,):
            raise ValueError("%s: weight / bias shapes" % name)
        out[name] = dict(w=w, w_scale=ws, w_zp=wz, bias=b.astype(np.float32), out_scale=float(s[12]),
                         out_zp=int(s[13]), stride=tuple(stride), padding=tuple(pad), kernel=tuple(ks))
    qm = root.state["quant"]
    sc, _ = ar.tensor(qm.state["scale"])
    zp, _ = ar.tensor(qm.state["zero_point"])
    out["input"] = dict(scale=float(sc.reshape(-1)[0]), zero_point=int(zp.reshape(-1)[0]))
    return out
