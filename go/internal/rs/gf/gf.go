// Package gf: GF(2^32-5) scalars and the byte<->symbol mapping of slime.
//
// Drop-in replacement for encryptio/slime's internal/rs/gf backed by
// libslime_rs.so (include/slime_rs.h): MapToGF, MapToGFWith and MapFromGF
// take and return host bytes, so the library runs them on the host cores in
// place on these slices (AVX2 passes over its copy pool; the GPU codec kernels
// serve device-resident buffers and the fused object entry points);
// MInverse and Raise are host scalars.
package gf

/*
#cgo LDFLAGS: -lslime_rs
#include <stdint.h>
#include <stdlib.h>
#include "slime_rs.h"
*/
import "C"

import (
	"fmt"
	"runtime"
	"unsafe"
)

const MaxVal = 1<<32 - 5

// Device is the GPU MapToGF / MapToGFWith / MapFromGF would use if the
// library's codec placement sends them to the GPU (slime_gf_codec_placement);
// -1 (C.SLIME_RS_ANY_DEVICE, the default) lets libslime_rs's device pool pick.
var Device = -1

const detailCap = 512

// call carries the device into one C call and that call's failure detail
// back out (see internal/rs: goroutines may change OS threads between cgo
// calls, so no thread-local state is read afterwards).
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

func (k call) check(rc C.int) {
	if rc != C.SLIME_RS_OK {
		panic(fmt.Sprintf("slime_rs: %s: %s", C.GoString(C.slime_rs_status_string(rc)), C.GoString(k.c.detail)))
	}
}

// MInverse returns in^(p-2) mod p: the multiplicative inverse of a nonzero element.
func MInverse(in uint32) uint32 { return uint32(C.slime_gf_minverse(C.uint32_t(in))) }

func Raise(x, n uint32) uint32 { return uint32(C.slime_gf_raise(C.uint32_t(x), C.uint32_t(n))) }

func bytesPtr(b []byte, p *runtime.Pinner) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	p.Pin(&b[0])
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

func wordsPtr(w []uint32, p *runtime.Pinner) *C.uint32_t {
	if len(w) == 0 {
		return nil
	}
	p.Pin(&w[0])
	return (*C.uint32_t)(unsafe.Pointer(&w[0]))
}

// MapToGF packs bytes big-endian into field symbols and picks the XOR mapping
// value that keeps every symbol below MaxVal (0, then 1<<31, then random).
func MapToGF(in []byte) (uint32, []uint32) {
	out := make([]uint32, (len(in)+3)/4)
	var pin runtime.Pinner
	defer pin.Unpin()
	var n C.uint32_t
	k := newCall()
	defer k.free()
	k.check(C.slime_gf_map_to_gf_ex(k.c, bytesPtr(in, &pin), C.uint64_t(len(in)), &n, wordsPtr(out, &pin)))
	return uint32(n), out
}

// MapToGFWith packs bytes with a mapping value MapToGF chose earlier.
func MapToGFWith(in []byte, n uint32) []uint32 {
	out := make([]uint32, (len(in)+3)/4)
	var pin runtime.Pinner
	defer pin.Unpin()
	k := newCall()
	defer k.free()
	k.check(C.slime_gf_map_to_gf_with_ex(k.c, bytesPtr(in, &pin), C.uint64_t(len(in)), C.uint32_t(n), wordsPtr(out, &pin)))
	return out
}

// MapFromGF undoes MapToGF: symbols XOR the mapping, emitted big-endian
// (4 bytes per symbol, so the result is a multiple of 4 bytes long).
func MapFromGF(inn uint32, inv []uint32) []byte {
	out := make([]byte, len(inv)*4)
	var pin runtime.Pinner
	defer pin.Unpin()
	k := newCall()
	defer k.free()
	k.check(C.slime_gf_map_from_gf_ex(k.c, C.uint32_t(inn), wordsPtr(inv, &pin), C.uint64_t(len(inv)), bytesPtr(out, &pin)))
	return out
}
