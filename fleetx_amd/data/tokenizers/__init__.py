from .gpt_tokenizer import GPTTokenizer, bytes_to_unicode  # noqa: F401
