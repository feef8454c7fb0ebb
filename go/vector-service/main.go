// Command vector-service serves rag/vector-service's HTTP API (GET /health,
// GET /collections, POST /upsert, POST /search on PORT, default 8082) from
// the MI355X engine through the vsearch cgo package, in place of the Qdrant
// server the reference dials (rag/vector-service/main.go:53-78). Callers
// (ingest-service storeVectors, retrieval-service searchVectorDB) see the
// same routes, JSON shapes, status codes and error prefixes.
//
// Environment:
//
//	PORT            listen port (8082)
//	VS_DEVICES      comma-separated HIP ordinals, one shard each ("0"); e.g.
//	                "0,1,2,3,4,5,6,7" row-shards every collection over a node
//	VS_PLACEMENT    with several devices: "stripes" (default, row shards) or
//	                "collections" (each collection whole on one device; calls
//	                for different collections run concurrently)
//	VS_DTYPE        storage of the collections: "f32" (the reference's) or "bf16"
//	VS_DIM          vector size (768: text-embedding-004)
//	VS_SNAPSHOT_DIR when set: restore at start-up from here
package main

import (
	"log"
	"net/http"
	"os"
	"strconv"
	"strings"

	"gorilla-rag/vsearch"
)

// The reference's hard-coded collections (main.go:85-87).
var collectionNames = []string{"regulatory_docs", "merchant_docs", "kyc_docs"}

func env(key, def string) string {
	if v := os.Getenv(key); v != "" {
		return v
	}
	return def
}

func openEngine() (*vsearch.Engine, error) {
	spec := env("VS_DEVICES", "0")
	var devs []int
	for _, f := range strings.Split(spec, ",") {
		d, err := strconv.Atoi(strings.TrimSpace(f))
		if err != nil {
			return nil, err
		}
		devs = append(devs, d)
	}
	if len(devs) == 1 {
		return vsearch.Open(devs[0])
	}
	if env("VS_PLACEMENT", "stripes") == "collections" {
		return vsearch.OpenPlaced(devs)
	}
	return vsearch.OpenShards(devs)
}

func main() {
	eng, err := openEngine()
	if err != nil {
		log.Fatalf("Failed to open the search engine: %v", err)
	}
	defer eng.Close()

	dtype := vsearch.DtypeF32
	if env("VS_DTYPE", "f32") == "bf16" {
		dtype = vsearch.DtypeBF16
	}
	dim, err := strconv.Atoi(env("VS_DIM", "768"))
	if err != nil || dim <= 0 {
		log.Fatalf("bad VS_DIM: %q", env("VS_DIM", "768"))
	}
	svc := newService(eng, uint32(dim), dtype)
	if err := svc.initCollections(collectionNames); err != nil {
		log.Printf("Warning: Failed to initialize collections: %v", err)
	}
	if dir := os.Getenv("VS_SNAPSHOT_DIR"); dir != "" {
		if err := svc.restore(dir); err != nil {
			log.Printf("Warning: restore from %s failed: %v", dir, err)
		}
	}

	mux := http.NewServeMux()
	mux.HandleFunc("/health", svc.health)
	mux.HandleFunc("/collections", svc.collections)
	mux.HandleFunc("/upsert", svc.upsert)
	mux.HandleFunc("/search", svc.search)

	port := env("PORT", "8082")
	log.Printf("Vector Service starting on port %s (engine: vsearch-hip, devices %s)", port,
		env("VS_DEVICES", "0"))
	log.Fatal(http.ListenAndServe(":"+port, mux))
}
