module github.com/cilium/cilium-amd/go

go 1.10
