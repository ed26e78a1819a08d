//go:build !(rocm && cgo)

package erasure

// Builds without the GPU codec (the default CGO_ENABLED=0 release builds,
// Dockerfile:20-22, builds.sh:8-20) keep the reference codec: after codec.go.diff its
// methods are named cpuEncode / cpuDecode, and these two forward to them, so the binary
// behaves exactly as before.

// Encode splits data into DataShards pieces and computes ParityShards parity shards.
func (c *Codec) Encode(data []byte, profile ErasureProfile) ([][]byte, error) {
	return c.cpuEncode(data, profile)
}

// Decode reconstructs the original data from shards (nil entries are missing).
func (c *Codec) Decode(shards [][]byte, profile ErasureProfile, originalSize int64) ([]byte, error) {
	return c.cpuDecode(shards, profile, originalSize)
}

// The pinned-buffer helpers of the GPU build (codec_rocm.go) exist here too, so callers
// compile on every build: there is no device, so HostBuffer and BodyBuffer return nil
// (read into heap buffers as before), FreeHostBuffer ignores its argument and DecodePinned
// is Decode.

// HostBuffer returns nil on builds without the GPU codec.
func HostBuffer(n int) []byte { return nil }

// BodyBuffer returns nil on builds without the GPU codec.
func BodyBuffer(size int, profile ErasureProfile) []byte { return nil }

// FreeHostBuffer does nothing on builds without the GPU codec.
func FreeHostBuffer(b []byte) {}

// DecodePinned is Decode on builds without the GPU codec.
func (c *Codec) DecodePinned(shards [][]byte, profile ErasureProfile, originalSize int64) ([]byte, error) {
	return c.cpuDecode(shards, profile, originalSize)
}
