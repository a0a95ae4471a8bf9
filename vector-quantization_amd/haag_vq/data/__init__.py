from .datasets import Dataset, load_dummy_dataset, load_local_dataset, load_dbpedia_openai_1536_100k

__all__ = ["Dataset", "load_dummy_dataset", "load_local_dataset", "load_dbpedia_openai_1536_100k"]
