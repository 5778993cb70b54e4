//go:build dgrep_gpu

// grep_gpu.go -- the drop-in grep plugin for bgilby59/distributed-grep with
// the Map body on MI355X through libdgrep.so (include/dgrep.h).
//
// Same exported symbols and types as the reference plugin
// (application/grep.go:13-40), looked up by main/worker_launch.go:21-34:
//   Map    func(string, string) []mapreduce.KeyValue
//   Reduce func(string, []string) string
// Only Map's body changes: the pattern is compiled once (dgrep_compile) instead
// of per line inside regexp.Match (grep.go:21), and the whole split is scanned
// on the GPU (dgrep_scan replaces grep.go:17-24); the KeyValues are rebuilt on
// the host exactly as grep.go:25-28 builds them.
//
// It declares the same package-level names as application/grep.go (pattern,
// Map, Reduce), so the two must never be compiled together. Either build
// (from the reference tree's root, this file copied to application/):
//   single file -- go ignores build constraints on files named on the command
//   line, and grep.go is not named:
//     go build -buildmode=plugin -o grep.so ./application/grep_gpu.go
//   or the package with tags -- after adding the line
//     //go:build !dgrep_gpu
//   (and a blank line) at the top of application/grep.go:
//     go build -tags dgrep_gpu -buildmode=plugin -o grep.so ./application
// with this repository's include/ and libdgrep.so on the cgo paths:
//     export CGO_CFLAGS="-I<repo>/include"
//     export CGO_LDFLAGS="-L<repo>/distributed-grep_amd -Wl,-rpath,<repo>/distributed-grep_amd"
// UNTESTED AS GO: there is no Go toolchain in this image or on the GPU box;
// tests/test_go_plugin.py checks the build constraints and top-level names of
// both files, and tests/abi_c/plugin_sequence.c runs the same call sequence
// from C on the GPU (tests/test_abi_c.py).
//
// Intended departures from grep.go (fail-stop, never a silent CPU path): a
// valid Go pattern outside the compiler's subset (DGREP_E_UNSUPPORTED /
// DGREP_E_TOO_LARGE) panics at the first Map, as does any HIP error; the
// worker dies and the coordinator's 10 s timeout re-assigns the task
// (map_reduce/coordinator.go:97-124). A pattern Go itself rejects is not a
// departure: it compiles to a match-nothing blob, as grep.go:21 drops the error.
//
// Device: dgrep_pick_device(-1) -- DGREP_DEVICE, else DGREP_WORKER_ID (or the
// process id) modulo the device count, so N worker processes on one node
// spread over its GPUs (the plugin never sees the RPC's WorkerID).
package main

/*
#cgo LDFLAGS: -ldgrep
#include <stdlib.h>
#include "dgrep.h"
*/
import "C"

import (
	"fmt"
	"os"
	"reflect"
	"runtime"
	"sync"
	"unsafe"

	"github.com/bgilby59/distributed-grep/mapreduce"
)

var pattern string = "" // grep.go:11; DGREP_PATTERN overrides (no RPC change)

var (
	once sync.Once
	ctx  *C.dgrep_ctx
)

func init() {
	if p, ok := os.LookupEnv("DGREP_PATTERN"); ok {
		pattern = p
	}
}

func setup() {
	runtime.LockOSThread() // the HIP current device is per OS thread
	defer runtime.UnlockOSThread()
	var blob unsafe.Pointer
	var n C.size_t
	var errbuf [256]C.char
	cp := C.CString(pattern)
	defer C.free(unsafe.Pointer(cp))
	if rc := C.dgrep_compile(cp, C.size_t(len(pattern)), &blob, &n, &errbuf[0], 256); rc != C.DGREP_OK {
		panic("dgrep_compile: " + C.GoString(&errbuf[0])) // unsupported construct: refuse, never guess
	}
	defer C.dgrep_blob_free(blob)
	var dev C.int
	if rc := C.dgrep_pick_device(-1, &dev); rc != C.DGREP_OK {
		panic(fmt.Sprintf("dgrep_pick_device: rc=%d (DGREP_DEVICE=%q)", int(rc), os.Getenv("DGREP_DEVICE")))
	}
	if rc := C.dgrep_open(dev, &ctx); rc != C.DGREP_OK {
		panic("dgrep_open: " + C.GoString(C.dgrep_last_error(ctx)))
	}
	if rc := C.dgrep_load_dfa(ctx, blob, n); rc != C.DGREP_OK {
		panic("dgrep_load_dfa: " + C.GoString(C.dgrep_last_error(ctx)))
	}
}

// Map: same signature and output as application/grep.go:13-36.
func Map(filename string, contents string) []mapreduce.KeyValue {
	once.Do(setup)
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	// Go 1.18 (go.mod:3) has no unsafe.StringData (1.20): the string header
	hdr := (*reflect.StringHeader)(unsafe.Pointer(&contents))
	var res C.dgrep_result
	// contents holds no Go pointers, so passing its bytes obeys the cgo rules;
	// the library borrows them only for the duration of the call.
	if rc := C.dgrep_scan(ctx, (*C.uint8_t)(unsafe.Pointer(hdr.Data)), C.size_t(len(contents)), &res); rc != C.DGREP_OK {
		panic("dgrep_scan: " + C.GoString(C.dgrep_last_error(ctx)))
	}
	defer C.dgrep_result_free(&res)
	n := int(res.count)
	kva := make([]mapreduce.KeyValue, 0, n)
	if n == 0 {
		return kva
	}
	lines := unsafe.Slice(res.line_no, n) // unsafe.Slice: Go 1.17+
	starts := unsafe.Slice(res.start, n)
	lens := unsafe.Slice(res.len, n)
	for i := 0; i < n; i++ {
		s := int(starts[i])
		k := fmt.Sprintf("%s (line number #%v)", filename, uint64(lines[i]))
		kva = append(kva, mapreduce.KeyValue{Key: k, Value: contents[s : s+int(lens[i])]})
	}
	return kva
}

// Reduce: unchanged (application/grep.go:38-40).
func Reduce(key string, values []string) string {
	return values[0]
}
