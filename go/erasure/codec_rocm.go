//go:build rocm && cgo

// GPU Reed-Solomon codec for CallFS on MI355X: the cgo side of the drop-in described in
// INTEGRATION.md. It replaces the two Codec methods of erasure/codec.go (Encode at
// :21-41, Decode at :45-78) on a `-tags rocm` build; NewCodec, ShardChecksum, the
// errors (errors.go) and ErasureProfile (metadata.go) stay the reference's own.
// codec.go.diff renames the reference's methods to cpuEncode / cpuDecode, which this
// file falls back to (and codec_cpu.go calls on every other build).
//
// Build: CGO_ENABLED=1 CGO_CFLAGS=-I<repo>/include CGO_LDFLAGS="-L<lib dir>" go build -tags rocm
package erasure

/*
#cgo LDFLAGS: -lcallfs_rs
#include <stdlib.h>
#include "callfs_rs.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"os"
	"runtime"
	"strconv"
	"sync"
	"unsafe"

	"github.com/klauspost/reedsolomon"
)

var (
	gpuOnce sync.Once
	gpuCtx  *C.rs_ctx // nil: no usable device, every call takes the CPU codec
	// CALLFS_ERASURE__GPU_MIN_BYTES: objects below this stay on the CPU codec
	// (INTEGRATION.md "when the GPU pays"). 64 MiB is where one GPU call passes one CPU
	// thread on the round-6 build (DESIGN.md §7.4 "CPU or GPU", tools/jobs.sh n1_r06,
	// profiles/r06/n1/): RS(10,4) 28.2 vs 20.0 GiB/s from pageable buffers and 33.0 through
	// pinned bodies (BodyBuffer), RS(4,2) 34.7 vs 29.3 through pinned bodies; at 16 MiB the
	// cache-resident CPU port leads (51-53 vs 20-33); one threshold for every profile.
	gpuMinBytes = envInt("CALLFS_ERASURE__GPU_MIN_BYTES", 64<<20)
)

func envInt(name string, def int) int {
	if v, err := strconv.Atoi(os.Getenv(name)); err == nil && v >= 0 {
		return v
	}
	return def
}

// device returns the process-wide context, created on first use. One rs_ctx serves
// every goroutine (all rs_* calls are thread-safe), like the shared *Codec at
// manager.go:60. CALLFS_ERASURE__GPU_MASK selects devices (bit d = HIP device d).
func device() *C.rs_ctx {
	gpuOnce.Do(func() {
		mask, _ := strconv.ParseUint(os.Getenv("CALLFS_ERASURE__GPU_MASK"), 0, 32)
		var c *C.rs_ctx
		if C.rs_init(&c, C.uint(mask)) == C.RS_OK {
			gpuCtx = c
		}
	})
	return gpuCtx
}

// upstreamErr maps an rs_* code to the reedsolomon error value the CPU codec would
// have returned, so errors.Is and the wrapped .Error() text match codec.go.
func upstreamErr(rc C.int) error {
	switch rc {
	case C.RS_E_SHORT_DATA:
		return reedsolomon.ErrShortData
	case C.RS_E_TOO_FEW_SHARDS:
		return reedsolomon.ErrTooFewShards
	case C.RS_E_NO_DATA:
		return reedsolomon.ErrShardNoData
	case C.RS_E_SHARD_SIZE:
		return reedsolomon.ErrShardSize
	case C.RS_E_SINGULAR:
		return reedsolomon.ErrSingular
	}
	return errors.New(C.GoString(C.rs_strerror(rc)))
}

// decodeErr maps rs_codec_decode / rs_reconstruct_batch codes the way Decode reports
// them: the erasure package's sentinels by identity (codec.go:63-65, :73-75), anything
// from Reconstruct inside its wrapper (codec.go:56).
func decodeErr(rc C.int) error {
	switch rc {
	case C.RS_OK:
		return nil
	case C.RS_E_CORRUPT:
		return ErrShardCorrupted
	case C.RS_E_INSUFFICIENT:
		return ErrInsufficientShards
	case C.RS_E_INVALID_PROFILE:
		return ErrInvalidProfile
	}
	return fmt.Errorf("erasure: reconstruction failed: %w", upstreamErr(rc))
}

// ---- pinned host buffers (zero-copy bodies) -------------------------------------------
//
// HostBuffer / BodyBuffer hand out page-locked host memory from rs_host_alloc as Go byte
// slices (C memory: cgo's pointer rules and runtime.Pinner do not apply to it, and the GC
// never moves it). When every shard of a call lies inside such buffers, the library runs
// the call zero-copy: H2D, kernels and D2H straight on these bytes, no CPU copy through its
// staging (include/callfs_rs.h rs_host_alloc; DESIGN.md §7.4, 38-45 GiB/s for objects of
// 10 MiB and up on one request thread). Upload bodies read into a BodyBuffer instead of
// io.ReadAll's heap slice (post_file_enhanced.go:125-127) and shards fetched into
// HostBuffers instead of io.ReadAll (manager.go:473,530) take that path. Release each with
// FreeHostBuffer; the context keeps freed buffers and hands them to later requests of a
// similar size (2 MiB granules), so page-locking is paid once, not per request.

// HostBuffer returns n bytes of pinned host memory, or nil when there is no device (read
// into a heap buffer then, as before).
func HostBuffer(n int) []byte {
	if n <= 0 || device() == nil {
		return nil
	}
	var p unsafe.Pointer
	if C.rs_host_alloc(gpuCtx, C.size_t(n), &p) != C.RS_OK {
		return nil
	}
	return unsafe.Slice((*byte)(p), n)
}

// BodyBuffer returns a pinned buffer of length size with capacity for the profile's n
// shards, n * ceil(size/k) bytes: read the upload body into it and pass it to Encode,
// whose Split (split below, as upstream's codec.go:31) then lays the data shards and the
// parity inside the one pinned allocation. nil when there is no device or the profile
// takes the CPU codec (k+m > 256).
func BodyBuffer(size int, profile ErasureProfile) []byte {
	k, m := profile.DataShards, profile.ParityShards
	if k < 1 || m < 1 || k+m > 256 || size <= 0 {
		return nil
	}
	S := (size + k - 1) / k
	b := HostBuffer((k + m) * S)
	if b == nil {
		return nil
	}
	return b[:size]
}

// FreeHostBuffer releases a HostBuffer or BodyBuffer (any reslice of it that starts at its
// first byte). A nil or heap slice is ignored.
func FreeHostBuffer(b []byte) {
	if cap(b) == 0 || gpuCtx == nil {
		return
	}
	C.rs_host_free(gpuCtx, unsafe.Pointer(unsafe.SliceData(b)))
}

// cArray is n pointer-sized C slots (cgo: a Go []*T passed to C may not hold Go
// pointers; a C array may, while each pointee is pinned).
type cArray struct {
	base unsafe.Pointer
	n    int
}

func newCArray(n int) cArray {
	return cArray{C.calloc(C.size_t(n), C.size_t(unsafe.Sizeof(uintptr(0)))), n}
}

func (a cArray) set(i int, p unsafe.Pointer) {
	*(*unsafe.Pointer)(unsafe.Add(a.base, i*int(unsafe.Sizeof(uintptr(0))))) = p
}

func (a cArray) at(i int) **C.uint8_t {
	return (**C.uint8_t)(unsafe.Add(a.base, i*int(unsafe.Sizeof(uintptr(0)))))
}

func (a cArray) free() { C.free(a.base) }

// Encode: Split in Go with upstream's aliasing and spare-capacity reuse (split below),
// parity on the GPU (rs_encode, codec.go:36). The object is never copied into a second
// host buffer.
func (c *Codec) Encode(data []byte, profile ErasureProfile) ([][]byte, error) {
	k, m := profile.DataShards, profile.ParityShards
	if k < 1 || m < 1 {
		return nil, ErrInvalidProfile // identity, codec_test.go:113,118
	}
	// Leopard GF(2^16) profiles, no device, or an object too small to amortise the
	// ~25 µs GPU round trip: the reference codec. (Empty objects fail in its Split with
	// the same wrapped error as here, whatever k+m is.)
	if k+m > 256 || len(data) < gpuMinBytes || len(data) == 0 || device() == nil {
		return c.cpuEncode(data, profile)
	}
	shards := split(data, k, m)
	S, n := len(shards[0]), k+m
	ptrs := newCArray(n)
	defer ptrs.free()
	var pin runtime.Pinner
	defer pin.Unpin()
	for i, s := range shards {
		pin.Pin(&s[0])
		ptrs.set(i, unsafe.Pointer(&s[0]))
	}
	if rc := C.rs_encode(gpuCtx, C.int(k), C.int(m), C.size_t(S), ptrs.at(0), ptrs.at(k)); rc != C.RS_OK {
		return nil, fmt.Errorf("erasure: failed to encode parity: %w", upstreamErr(rc))
	}
	return shards, nil
}

// split lays out the n shards as upstream Split does (codec.go:31): S = ceil(len/k);
// spare capacity of data (up to n*S bytes) is zeroed past len and used in place;
// every shard lying entirely inside that extent is a sub-slice of data (the parity too
// when the capacity reaches it), and the rest are fresh zeroed buffers that receive
// the partial shard's bytes.
func split(data []byte, k, m int) [][]byte {
	n := k + m
	S := (len(data) + k - 1) / k
	need := n * S
	ext := data
	if cap(data) > len(data) {
		ext = data[:min(cap(data), need)]
		clear(ext[len(data):])
	}
	full := len(ext) / S
	shards := make([][]byte, n)
	for i := 0; i < full && i < n; i++ {
		shards[i] = ext[i*S : (i+1)*S : (i+1)*S]
	}
	if full < n {
		pad := make([]byte, (n-full)*S)
		copy(pad, ext[full*S:]) // the partial shard (zeros past len(data) stay zero)
		for i := full; i < n; i++ {
			shards[i] = pad[(i-full)*S : (i-full+1)*S : (i-full+1)*S]
		}
	}
	return shards
}

// Decode: Reconstruct + Verify + join + trim in one call (rs_codec_decode).
//
// Like upstream Reconstruct, nil or empty entries of shards are filled with the
// reconstructed shards (reusing an entry's capacity when it holds S bytes). They are
// filled only once Reconstruct has succeeded: the buffers are prepared in a private
// copy of the slice and handed over after the call, so a call failing with
// ErrTooFewShards / ErrShardSize / ErrShardNoData leaves the caller's slice exactly as
// it was (codec_test.go:65-88).
func (c *Codec) Decode(shards [][]byte, profile ErasureProfile, originalSize int64) ([]byte, error) {
	return c.decode(shards, profile, originalSize, false)
}

// DecodePinned is Decode for shards fetched into HostBuffers (manager.go:473,530 reading
// into HostBuffer(S) instead of io.ReadAll): the reconstructed entries it fills and the
// object it returns are HostBuffers too, so the whole call runs zero-copy. The caller
// releases the returned object and every shard entry with FreeHostBuffer once the response
// is written -- on the ErrShardCorrupted and ErrInsufficientShards paths as well: there
// Reconstruct has run and the nil entries are filled with HostBuffers, as upstream fills
// them (codec.go:55), so the caller owns and frees them. Every other error leaves the
// caller's slice untouched and frees what the call allocated. Without a device it is
// Decode (heap buffers, FreeHostBuffer ignores them).
// Not in the reference API: an addition for servers that read into pinned buffers.
func (c *Codec) DecodePinned(shards [][]byte, profile ErasureProfile, originalSize int64) ([]byte, error) {
	return c.decode(shards, profile, originalSize, true)
}

func (c *Codec) decode(shards [][]byte, profile ErasureProfile, originalSize int64, pinned bool) ([]byte, error) {
	k, m := profile.DataShards, profile.ParityShards
	if k < 1 || m < 1 {
		return nil, ErrInvalidProfile
	}
	n := k + m
	if n > 256 || originalSize < int64(gpuMinBytes) || device() == nil {
		return c.cpuDecode(shards, profile, originalSize)
	}
	alloc := func(size int) []byte { return make([]byte, size) }
	var owned [][]byte // HostBuffers this call allocated, released unless handed over
	if pinned {
		alloc = func(size int) []byte {
			if b := HostBuffer(size); b != nil {
				owned = append(owned, b)
				return b
			}
			return make([]byte, size)
		}
	}
	if len(shards) != n {
		return nil, fmt.Errorf("erasure: reconstruction failed: %w", reedsolomon.ErrTooFewShards)
	}
	S := 0
	for _, s := range shards {
		if len(s) != 0 {
			S = len(s)
			break
		}
	}
	bufs := make([][]byte, n)
	copy(bufs, shards)
	ptrs := newCArray(n)
	defer ptrs.free()
	lens := (*C.size_t)(C.calloc(C.size_t(n), C.size_t(unsafe.Sizeof(C.size_t(0)))))
	defer C.free(unsafe.Pointer(lens))
	lensAt := func(i int) *C.size_t {
		return (*C.size_t)(unsafe.Add(unsafe.Pointer(lens), i*int(unsafe.Sizeof(C.size_t(0)))))
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	for i := range bufs {
		*lensAt(i) = C.size_t(len(bufs[i]))
		if len(bufs[i]) == 0 && S > 0 {
			if cap(bufs[i]) >= S {
				bufs[i] = bufs[i][:S]
			} else {
				bufs[i] = alloc(S)
			}
		}
		if len(bufs[i]) > 0 {
			pin.Pin(&bufs[i][0])
			ptrs.set(i, unsafe.Pointer(&bufs[i][0]))
		}
	}
	buf := alloc(int(originalSize))
	var out *C.uint8_t
	if originalSize > 0 {
		pin.Pin(&buf[0])
		out = (*C.uint8_t)(unsafe.Pointer(&buf[0]))
	}
	rc := C.rs_codec_decode(gpuCtx, C.int(k), C.int(m), ptrs.at(0), lens, out, C.int64_t(originalSize))
	handed := map[*byte]bool{}
	switch rc {
	case C.RS_OK, C.RS_E_CORRUPT, C.RS_E_INSUFFICIENT:
		// Reconstruct ran: upstream has filled the nil entries by now (codec.go:55)
		for i := range shards {
			if len(shards[i]) == 0 {
				shards[i] = bufs[i]
				handed[unsafe.SliceData(bufs[i])] = true
			}
		}
	}
	if rc == C.RS_OK {
		handed[unsafe.SliceData(buf)] = true
	}
	for _, b := range owned { // pinned buffers the caller did not receive
		if !handed[unsafe.SliceData(b)] {
			FreeHostBuffer(b)
		}
	}
	if rc != C.RS_OK {
		return nil, decodeErr(rc)
	}
	return buf, nil
}

// RepairBatch reconstructs the missing shards of many objects in one call
// (rs_reconstruct_batch), e.g. every object that lost a shard with a node. objs[b] is
// object b's n shards (nil or empty = missing). Each object's missing entries are
// filled only when that object succeeded; errs[b] is what Decode would report for it
// (Verify of the present parity beyond the first k included). Not in the reference
// API: an addition for bulk callers, no existing caller changes.
func (c *Codec) RepairBatch(objs [][][]byte, profile ErasureProfile) []error {
	k, m := profile.DataShards, profile.ParityShards
	errs := make([]error, len(objs))
	if k < 1 || m < 1 {
		for b := range errs {
			errs[b] = ErrInvalidProfile
		}
		return errs
	}
	n := k + m
	if len(objs) == 0 {
		return errs
	}
	if n > 256 || device() == nil {
		for b, shards := range objs {
			errs[b] = cpuRepair(shards, k, m)
		}
		return errs
	}
	bufs := make([][][]byte, len(objs))
	ptrs := newCArray(len(objs) * n)
	defer ptrs.free()
	lens := make([]C.size_t, len(objs)*n) // Go memory without Go pointers: may be passed
	status := make([]C.int, len(objs))
	var pin runtime.Pinner
	defer pin.Unpin()
	for b, shards := range objs {
		if len(shards) != n {
			errs[b] = fmt.Errorf("erasure: reconstruction failed: %w", reedsolomon.ErrTooFewShards)
			continue // all lens 0 and no pointers: the stripe reports RS_E_NO_DATA, ignored
		}
		S := 0
		for _, s := range shards {
			if len(s) > 0 {
				S = len(s)
				break
			}
		}
		bufs[b] = make([][]byte, n)
		copy(bufs[b], shards)
		for i, s := range bufs[b] {
			lens[b*n+i] = C.size_t(len(s))
			if len(s) == 0 && S > 0 {
				s = make([]byte, S)
				bufs[b][i] = s
			}
			if len(s) > 0 {
				pin.Pin(&s[0])
				ptrs.set(b*n+i, unsafe.Pointer(&s[0]))
			}
		}
	}
	rc := C.rs_reconstruct_batch(gpuCtx, C.int(k), C.int(m), C.int(len(objs)), ptrs.at(0),
		&lens[0], 1, &status[0])
	stripeArg := false // RS_E_ARG is per-stripe only when some stripe reports it
	for _, st := range status {
		stripeArg = stripeArg || st == C.RS_E_ARG
	}
	switch {
	case rc == C.RS_OK, rc == C.RS_E_CORRUPT, rc == C.RS_E_TOO_FEW_SHARDS,
		rc == C.RS_E_SHARD_SIZE, rc == C.RS_E_NO_DATA, rc == C.RS_E_ARG && stripeArg:
		// per-stripe statuses are valid (RS_E_ARG: a stripe with a nil present entry)
	default: // a call-level error: no status was written
		for b := range errs {
			if errs[b] == nil {
				errs[b] = decodeErr(rc)
			}
		}
		return errs
	}
	for b, shards := range objs {
		if errs[b] != nil {
			continue
		}
		st := status[b]
		if st == C.RS_OK || st == C.RS_E_CORRUPT {
			for i := range shards {
				if len(shards[i]) == 0 {
					shards[i] = bufs[b][i]
				}
			}
		}
		errs[b] = decodeErr(st)
	}
	return errs
}

// cpuRepair is RepairBatch's per-object CPU form: upstream Reconstruct + Verify.
func cpuRepair(shards [][]byte, k, m int) error {
	enc, err := reedsolomon.New(k, m)
	if err != nil {
		return fmt.Errorf("erasure: failed to create decoder: %w", err)
	}
	if err := enc.Reconstruct(shards); err != nil {
		return fmt.Errorf("erasure: reconstruction failed: %w", err)
	}
	ok, err := enc.Verify(shards)
	if err != nil {
		return fmt.Errorf("erasure: verification failed: %w", err)
	}
	if !ok {
		return ErrShardCorrupted
	}
	return nil
}
