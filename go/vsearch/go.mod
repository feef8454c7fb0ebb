module gorilla-rag/vsearch

go 1.21
