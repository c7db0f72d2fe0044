// Package gf: GF(2^32-5) scalars and the byte<->symbol mapping of slime.
//
// Drop-in replacement for encryptio/slime's internal/rs/gf backed by the
// MI355X codec in libslime_rs.so (include/slime_rs.h): MapToGF, MapToGFWith
// and MapFromGF run on the GPU; MInverse and Raise are host scalars.
package gf

/*
#cgo LDFLAGS: -lslime_rs
#include <stdint.h>
#include "slime_rs.h"
*/
import "C"

import (
	"fmt"
	"runtime"
	"unsafe"
)

const MaxVal = 1<<32 - 5

func check(rc C.int) {
	if rc != C.SLIME_RS_OK {
		panic(fmt.Sprintf("slime_rs: %s: %s", C.GoString(C.slime_rs_status_string(rc)), C.GoString(C.slime_rs_last_error())))
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
	check(C.slime_gf_map_to_gf(bytesPtr(in, &pin), C.uint64_t(len(in)), &n, wordsPtr(out, &pin)))
	return uint32(n), out
}

// MapToGFWith packs bytes with a mapping value MapToGF chose earlier.
func MapToGFWith(in []byte, n uint32) []uint32 {
	out := make([]uint32, (len(in)+3)/4)
	var pin runtime.Pinner
	defer pin.Unpin()
	check(C.slime_gf_map_to_gf_with(bytesPtr(in, &pin), C.uint64_t(len(in)), C.uint32_t(n), wordsPtr(out, &pin)))
	return out
}

// MapFromGF undoes MapToGF: symbols XOR the mapping, emitted big-endian
// (4 bytes per symbol, so the result is a multiple of 4 bytes long).
func MapFromGF(inn uint32, inv []uint32) []byte {
	out := make([]byte, len(inv)*4)
	var pin runtime.Pinner
	defer pin.Unpin()
	check(C.slime_gf_map_from_gf(C.uint32_t(inn), wordsPtr(inv, &pin), C.uint64_t(len(inv)), bytesPtr(out, &pin)))
	return out
}
