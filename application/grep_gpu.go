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
// Build (in the reference tree, next to application/grep.go):
//   go build -buildmode=plugin -o grep.so ./application
// with this repository's include/ and distributed-grep_amd/libdgrep.so on the
// cgo paths below. There is no Go toolchain in this image or on the GPU box;
// tests/abi_c/plugin_sequence.c runs the same call sequence from C and is
// tested on the GPU (tests/test_abi_c.py).
package main

/*
#cgo CFLAGS: -I${SRCDIR}/../include
#cgo LDFLAGS: -L${SRCDIR}/../distributed-grep_amd -ldgrep -Wl,-rpath,${SRCDIR}/../distributed-grep_amd
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
	if rc := C.dgrep_open(0, &ctx); rc != C.DGREP_OK {
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
	lines := (*[1 << 40]C.uint64_t)(unsafe.Pointer(res.line_no))[:n:n]
	starts := (*[1 << 40]C.uint64_t)(unsafe.Pointer(res.start))[:n:n]
	lens := (*[1 << 40]C.uint32_t)(unsafe.Pointer(res.len))[:n:n]
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
