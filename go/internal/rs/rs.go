// Package rs implements Reed-Solomon erasure coding using Vandermonde
// coefficient matricies over GF(2^32-5).
//
// This is the drop-in replacement for encryptio/slime's internal/rs: the same
// exported API (CreateParity, RecoverData, ParityMatrix, ParityMatrixCached)
// and the unexported helpers the reference's own tests call
// (vandermondeMatrix, solveSubIdentity, cloneMatrix, invertMatrix), backed by
// the MI355X (gfx950) HIP implementation in libslime_rs.so through its C-ABI
// (include/slime_rs.h).  Panics carry the reference's exact messages.
//
// Build: `make` at the slime-rs-mi355x repo root, then point cgo at it, e.g.
//   CGO_CFLAGS=-I$SLIME_RS/include CGO_LDFLAGS="-L$SLIME_RS/slime_amd/lib -lslime_rs"
package rs

/*
#cgo LDFLAGS: -lslime_rs
#include <stdint.h>
#include <stdlib.h>
#include "slime_rs.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"sync"
	"unsafe"
)

// Device is the GPU the data-path calls of this package run on.  The default,
// C.SLIME_RS_ANY_DEVICE (-1), lets libslime_rs's device pool give each call
// the visible GPU with the fewest calls in flight, so concurrent goroutines
// (HTTP requests, main.go:107-109; scrubbers, multi.go:54-58) spread over
// every GPU of the node.  Additive: the reference has no device to choose.
var Device = -1

const detailCap = 512

// call is one C-allocated slime_rs_call_t with its detail buffer.  The
// device goes in with the call and the failure detail of THAT call comes
// back in the buffer, so nothing depends on which OS thread cgo runs the
// call on: a goroutine may move between threads from one C call to the next,
// which makes the library's thread-local state (the last-error string, the
// per-thread device choice) unusable from Go.
type call struct{ c *C.slime_rs_call_t }

func newCall() call {
	size := C.size_t(unsafe.Sizeof(C.slime_rs_call_t{}))
	c := (*C.slime_rs_call_t)(C.calloc(1, size+detailCap))
	c.device = C.int(Device)
	c.detail = (*C.char)(unsafe.Add(unsafe.Pointer(c), size))
	c.detail_cap = detailCap
	return call{c}
}

func (k call) free() { C.free(unsafe.Pointer(k.c)) }

// raise turns the status of the call made with k into the reference's panic.
func (k call) raise(rc C.int) {
	if rc == C.SLIME_RS_OK {
		return
	}
	// Codes 1..7: the reference's own panic strings (static, thread-free).
	if rc >= 1 && rc <= 7 {
		panic(C.GoString(C.slime_rs_status_string(rc)))
	}
	detail := C.GoString(k.c.detail)
	if rc == C.SLIME_RS_ERR_INDEX_RANGE && detail != "" {
		panic(detail) // Go's runtime index-out-of-range text, as produced by this call
	}
	panic(fmt.Sprintf("slime_rs: %s: %s", C.GoString(C.slime_rs_status_string(rc)), detail))
}

// vectors pins the backing arrays of vs and returns a C array of their data
// pointers plus their lengths (cgo forbids Go pointers in C memory unless
// pinned; runtime.Pinner, Go >= 1.21).  Call free() when C has returned.
type vectors struct {
	ptrs   **C.uint32_t
	lens   *C.uint64_t
	pinner runtime.Pinner
}

func marshal(vs [][]uint32) *vectors {
	n := len(vs)
	if n == 0 {
		n = 1
	}
	m := &vectors{
		ptrs: (**C.uint32_t)(C.calloc(C.size_t(n), C.size_t(unsafe.Sizeof(uintptr(0))))),
		lens: (*C.uint64_t)(C.calloc(C.size_t(n), 8)),
	}
	ps := unsafe.Slice(m.ptrs, n)
	ls := unsafe.Slice(m.lens, n)
	for i, v := range vs {
		ls[i] = C.uint64_t(len(v))
		if cap(v) > 0 {
			p := &v[:1][0]
			m.pinner.Pin(p)
			ps[i] = (*C.uint32_t)(unsafe.Pointer(p))
		}
	}
	return m
}

func (m *vectors) free() {
	m.pinner.Unpin()
	C.free(unsafe.Pointer(m.ptrs))
	C.free(unsafe.Pointer(m.lens))
}

func matrixFromC(p *C.uint32_t, rows, cols int) [][]uint32 {
	underlying := make([]uint32, rows*cols)
	if rows*cols > 0 {
		copy(underlying, unsafe.Slice((*uint32)(unsafe.Pointer(p)), rows*cols))
	}
	m := make([][]uint32, rows)
	for i := range m {
		m[i] = underlying[i*cols : (i+1)*cols : (i+1)*cols]
	}
	return m
}

func flatten(m [][]uint32) []uint32 {
	if len(m) == 0 {
		return nil
	}
	out := make([]uint32, 0, len(m)*len(m[0]))
	for _, r := range m {
		out = append(out, r...)
	}
	return out
}

// CreateParity returns code row `index` of the equal-length data vectors
// (internal/rs/vector.go:18), computed on the GPU; `out` is reused when its
// capacity allows.
func CreateParity(data [][]uint32, index int, out []uint32) []uint32 {
	for i := 1; i < len(data); i++ {
		if len(data[i]) != len(data[0]) {
			panic("CreateParity called on data chunks of varying length")
		}
	}
	if len(data) == 0 {
		_ = data[0] // the reference's index-out-of-range panic
	}
	if cap(out) < len(data[0]) {
		out = make([]uint32, len(data[0]))
	} else {
		out = out[:len(data[0])]
	}
	m := marshal(data)
	defer m.free()
	var op *C.uint32_t
	if len(out) > 0 {
		var pin runtime.Pinner
		pin.Pin(&out[0])
		defer pin.Unpin()
		op = (*C.uint32_t)(unsafe.Pointer(&out[0]))
	}
	k := newCall()
	defer k.free()
	k.raise(C.slime_rs_create_parity_ex(k.c, m.ptrs, m.lens, C.int(len(data)), C.int(index), op))
	return out
}

// CreateParities computes every parity row total-len(data)..total-1 in one GPU
// pass (multi_store.go:528-531 calls CreateParity once per row instead).
func CreateParities(data [][]uint32, total int) [][]uint32 {
	for i := 1; i < len(data); i++ {
		if len(data[i]) != len(data[0]) {
			panic("CreateParity called on data chunks of varying length")
		}
	}
	outs := make([][]uint32, total-len(data))
	for i := range outs {
		outs[i] = make([]uint32, len(data[0]))
	}
	m := marshal(data)
	defer m.free()
	o := marshal(outs)
	defer o.free()
	k := newCall()
	defer k.free()
	k.raise(C.slime_rs_create_parities_ex(k.c, m.ptrs, m.lens, C.int(len(data)), C.int(total), o.ptrs))
	return outs
}

// RecoverData rebuilds all data vectors from exactly len(chunks) surviving code
// rows with the given indices (internal/rs/vector.go:50): the erased data rows
// on the GPU, the surviving ones (unit rows of the inverse) on the host.
func RecoverData(chunks [][]uint32, indices []int) [][]uint32 {
	if len(chunks) != len(indices) {
		panic("RecoverData: len(chunks) != len(indices)")
	}
	if len(chunks) == 0 {
		panic("RecoverData: len(chunks) == 0")
	}
	data := make([][]uint32, len(chunks))
	for i := range data {
		data[i] = make([]uint32, len(chunks[0]))
	}
	idx := (*C.int)(C.calloc(C.size_t(len(indices)), C.size_t(unsafe.Sizeof(C.int(0)))))
	defer C.free(unsafe.Pointer(idx))
	is := unsafe.Slice(idx, len(indices))
	for i, v := range indices {
		is[i] = C.int(v)
	}
	m := marshal(chunks)
	defer m.free()
	o := marshal(data)
	defer o.free()
	k := newCall()
	defer k.free()
	k.raise(C.slime_rs_recover_data_ex(k.c, m.ptrs, m.lens, C.int(len(chunks)), idx, C.int(len(indices)), o.ptrs))
	return data
}

// vandermondeMatrix: (d+p) x d, entry [i][j] = (j+1)^i mod p (host, exact).
func vandermondeMatrix(d, p int) [][]uint32 {
	buf := make([]C.uint32_t, (d+p)*d+1)
	k := newCall()
	defer k.free()
	k.raise(C.slime_rs_vandermonde_matrix_ex(k.c, C.int(d), C.int(p), &buf[0]))
	return matrixFromC(&buf[0], d+p, d)
}

// ParityMatrix: the systematic (d+p) x d code matrix (identity on top; any d
// rows invertible), computed exactly on the host by libslime_rs.
func ParityMatrix(d, p int) [][]uint32 {
	buf := make([]C.uint32_t, (d+p)*d+1)
	k := newCall()
	defer k.free()
	k.raise(C.slime_rs_parity_matrix_ex(k.c, C.int(d), C.int(p), &buf[0]))
	return matrixFromC(&buf[0], d+p, d)
}

var parityCache sync.Map // struct{ d, p int } -> [][]uint32

// ParityMatrixCached: process-wide memo of ParityMatrix; callers must not
// modify the returned rows (shared, as in the reference).
func ParityMatrixCached(d, p int) [][]uint32 {
	key := struct{ d, p int }{d, p}
	if v, ok := parityCache.Load(key); ok {
		return v.([][]uint32)
	}
	v, _ := parityCache.LoadOrStore(key, ParityMatrix(d, p))
	return v.([][]uint32)
}

// solveSubIdentity column-reduces m in place so its top square block becomes
// the identity; singular input panics with the reference's message.
func solveSubIdentity(m [][]uint32) {
	flat := flatten(m)
	k := newCall()
	defer k.free()
	rc := C.slime_rs_solve_sub_identity_ex(k.c, (*C.uint32_t)(unsafe.Pointer(&flat[0])), C.int(len(m)), C.int(len(m[0])))
	for i := range m {
		copy(m[i], flat[i*len(m[0]):(i+1)*len(m[0])])
	}
	k.raise(rc)
}

// cloneMatrix deep-copies m into rows that share one backing array.
func cloneMatrix(m [][]uint32) [][]uint32 {
	flat := flatten(m)
	n := make([][]uint32, len(m))
	off := 0
	for i, r := range m {
		n[i] = flat[off : off+len(r) : off+len(r)]
		off += len(r)
	}
	return n
}

func invertMatrix(m [][]uint32) [][]uint32 {
	flat := flatten(m)
	d := len(m[0])
	inv := make([]C.uint32_t, d*d)
	k := newCall()
	defer k.free()
	k.raise(C.slime_rs_invert_matrix_ex(k.c, (*C.uint32_t)(unsafe.Pointer(&flat[0])), C.int(d), &inv[0]))
	return matrixFromC(&inv[0], d, d)
}

// chunkBuffers allocates the total chunk slices of a writeChunks call.  A data
// chunk that lies wholly inside the object is the object's own bytes
// (MapFromGF(m, MapToGF(x)) = x, map.go:15-33,103-113), so it is returned as a
// capacity-limited subslice of data and the library skips its copy; the rest
// are fresh.  The caller must not modify data while it uses the chunks, which
// writeChunks never does (the request body is read-only from there on).
func chunkBuffers(data []byte, need, total, cb int) [][]byte {
	chunks := make([][]byte, total)
	for i := range chunks {
		if i < need && cb > 0 && (i+1)*cb <= len(data) {
			chunks[i] = data[i*cb : (i+1)*cb : (i+1)*cb]
		} else {
			chunks[i] = make([]byte, cb)
		}
	}
	return chunks
}

// WriteChunks is the data path of Multi.writeChunks
// (internal/store/multi/multi_store.go:526-531 and :554) in one GPU pass:
// gf.MapToGF, splitVector, CreateParity for every parity row, gf.MapFromGF per
// part.  It returns MappingValue and the total chunks as written to stores
// (whole data chunks alias data, see chunkBuffers).
// Not part of the reference's rs API: it lets writeChunks replace its
// per-row CreateParity loop and per-part MapFromGF calls (see INTEGRATION.md).
func WriteChunks(data []byte, need, total int) (uint32, [][]byte) {
	cb := int(C.slime_rs_chunk_size(C.uint64_t(len(data)), C.int(need)))
	chunks := chunkBuffers(data, need, total, cb)
	ptrs := (**C.uint8_t)(C.calloc(C.size_t(total+1), C.size_t(unsafe.Sizeof(uintptr(0)))))
	defer C.free(unsafe.Pointer(ptrs))
	ps := unsafe.Slice(ptrs, total+1)
	var pinner runtime.Pinner
	defer pinner.Unpin()
	for i := range chunks {
		if cb > 0 {
			pinner.Pin(&chunks[i][0])
			ps[i] = (*C.uint8_t)(unsafe.Pointer(&chunks[i][0]))
		}
	}
	var in *C.uint8_t
	if len(data) > 0 {
		pinner.Pin(&data[0])
		in = (*C.uint8_t)(unsafe.Pointer(&data[0]))
	}
	var mapping C.uint32_t
	k := newCall()
	defer k.free()
	k.raise(C.slime_rs_write_chunks_ex(k.c, in, C.uint64_t(len(data)), C.int(need), C.int(total), ptrs, &mapping))
	return uint32(mapping), chunks
}

// ReconstructObject is the slow path of Multi.reconstruct
// (multi_store.go:215-241): from exactly need surviving chunks (equal length)
// and their indices, gf.MapToGFWith + RecoverData + gf.MapFromGF, truncated to
// size.  Panics as RecoverData does for bad indices.
func ReconstructObject(chunks [][]byte, indices []int, mapping uint32, size int) []byte {
	n := len(chunks)
	if n != len(indices) {
		panic("RecoverData: len(chunks) != len(indices)")
	}
	cb := 0
	if n > 0 {
		cb = len(chunks[0])
	}
	ptrs := (**C.uint8_t)(C.calloc(C.size_t(n+1), C.size_t(unsafe.Sizeof(uintptr(0)))))
	defer C.free(unsafe.Pointer(ptrs))
	idx := (*C.int)(C.calloc(C.size_t(n+1), C.size_t(unsafe.Sizeof(C.int(0)))))
	defer C.free(unsafe.Pointer(idx))
	ps, is := unsafe.Slice(ptrs, n+1), unsafe.Slice(idx, n+1)
	var pinner runtime.Pinner
	defer pinner.Unpin()
	for i, c := range chunks {
		if len(c) < cb {
			panic(fmt.Sprintf("runtime error: index out of range [%d] with length %d", len(c), len(c)))
		}
		if cb > 0 {
			pinner.Pin(&c[0])
			ps[i] = (*C.uint8_t)(unsafe.Pointer(&c[0]))
		}
		is[i] = C.int(indices[i])
	}
	out := make([]byte, size, size+16)
	var op *C.uint8_t
	if size > 0 {
		pinner.Pin(&out[0])
		op = (*C.uint8_t)(unsafe.Pointer(&out[0]))
	}
	k := newCall()
	defer k.free()
	k.raise(C.slime_rs_reconstruct_ex(k.c, ptrs, idx, C.int(n), C.uint64_t(cb), C.uint32_t(mapping), C.uint64_t(size), op))
	return out
}

// WriteChunksDigest is WriteChunks plus every chunk's SHA-256: the value each
// of writeChunks' per-chunk goroutines computes with store.DataV
// (internal/store/store.go:104-110, multi_store.go:554-556), hashed by
// libslime_rs on its host threads while the GPU pipeline still runs.  A
// caller builds store.CASV{Present: true, SHA256: sums[i], Data: chunks[i]}
// instead of calling store.DataV.
func WriteChunksDigest(data []byte, need, total int) (uint32, [][]byte, [][32]byte) {
	cb := int(C.slime_rs_chunk_size(C.uint64_t(len(data)), C.int(need)))
	chunks := chunkBuffers(data, need, total, cb)
	sums := make([][32]byte, total+1)
	ptrs := (**C.uint8_t)(C.calloc(C.size_t(total+1), C.size_t(unsafe.Sizeof(uintptr(0)))))
	defer C.free(unsafe.Pointer(ptrs))
	ps := unsafe.Slice(ptrs, total+1)
	var pinner runtime.Pinner
	defer pinner.Unpin()
	for i := range chunks {
		if cb > 0 {
			pinner.Pin(&chunks[i][0])
			ps[i] = (*C.uint8_t)(unsafe.Pointer(&chunks[i][0]))
		}
	}
	var in *C.uint8_t
	if len(data) > 0 {
		pinner.Pin(&data[0])
		in = (*C.uint8_t)(unsafe.Pointer(&data[0]))
	}
	pinner.Pin(&sums[0])
	var mapping C.uint32_t
	k := newCall()
	defer k.free()
	k.raise(C.slime_rs_write_chunks_digest_ex(k.c, in, C.uint64_t(len(data)), C.int(need), C.int(total), ptrs, &mapping,
		(*C.uint8_t)(unsafe.Pointer(&sums[0][0])), nil))
	return uint32(mapping), chunks, sums[:total]
}

// ErrBadHash mirrors multi's ErrBadHash (multi_store.go:26).
var ErrBadHash = errors.New("bad checksum after reconstruction")

// ReconstructObjectVerified is ReconstructObject followed by reconstruct's
// verify step (multi_store.go:244-249): the rebuilt object's SHA-256 must
// equal sum (meta.File.SHA256), else ErrBadHash.
func ReconstructObjectVerified(chunks [][]byte, indices []int, mapping uint32, size int, sum [32]byte) ([]byte, error) {
	n := len(chunks)
	if n != len(indices) {
		panic("RecoverData: len(chunks) != len(indices)")
	}
	cb := 0
	if n > 0 {
		cb = len(chunks[0])
	}
	ptrs := (**C.uint8_t)(C.calloc(C.size_t(n+1), C.size_t(unsafe.Sizeof(uintptr(0)))))
	defer C.free(unsafe.Pointer(ptrs))
	idx := (*C.int)(C.calloc(C.size_t(n+1), C.size_t(unsafe.Sizeof(C.int(0)))))
	defer C.free(unsafe.Pointer(idx))
	ps, is := unsafe.Slice(ptrs, n+1), unsafe.Slice(idx, n+1)
	var pinner runtime.Pinner
	defer pinner.Unpin()
	for i, c := range chunks {
		if len(c) < cb {
			panic(fmt.Sprintf("runtime error: index out of range [%d] with length %d", len(c), len(c)))
		}
		if cb > 0 {
			pinner.Pin(&c[0])
			ps[i] = (*C.uint8_t)(unsafe.Pointer(&c[0]))
		}
		is[i] = C.int(indices[i])
	}
	out := make([]byte, size, size+16)
	var op *C.uint8_t
	if size > 0 {
		pinner.Pin(&out[0])
		op = (*C.uint8_t)(unsafe.Pointer(&out[0]))
	}
	pinner.Pin(&sum)
	k := newCall()
	defer k.free()
	rc := C.slime_rs_reconstruct_verify_ex(k.c, ptrs, idx, C.int(n), C.uint64_t(cb), C.uint32_t(mapping), C.uint64_t(size),
		op, (*C.uint8_t)(unsafe.Pointer(&sum[0])))
	if rc == C.SLIME_RS_ERR_BAD_HASH {
		return nil, ErrBadHash
	}
	k.raise(rc)
	return out, nil
}

